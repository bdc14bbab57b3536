#!/usr/bin/env python3
"""Generate the JPEG decode fixtures (tests/golden/jpeg_fixtures.npz).

Each case is a baseline JPEG encoded here by PIL (libjpeg-turbo) from a seeded
synthetic frame (mcmtt_opticalflow_amd/synth.py colourised) and PIL's own
decode of it, in OpenCV's BGR order: the fixtures pin oracle/jpeg_oracle.c
and the device decoder (include/psn_jpeg.h) to libjpeg-turbo's islow IDCT,
fancy upsampling and colour tables. Run: python tests/golden/make_jpeg_golden.py
"""
import io
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mcmtt_opticalflow_amd import synth  # noqa: E402

CASES = [  # (name, width, height, PIL save options)
    ("420_q75", 97, 61, dict(quality=75, subsampling=2)),
    ("422_q90", 97, 61, dict(quality=90, subsampling=1)),
    ("444_q95", 97, 61, dict(quality=95, subsampling=0)),
    ("420_q30_rst3", 97, 61, dict(quality=30, subsampling=2, restart_marker_blocks=3)),
    ("420_q85_rstrow", 320, 240, dict(quality=85, subsampling=2, restart_marker_rows=1)),
    ("422_q60_rst5", 131, 97, dict(quality=60, subsampling=1, restart_marker_blocks=5)),
    ("gray_q80", 77, 45, dict(quality=80)),
    ("420_tiny", 5, 3, dict(quality=90, subsampling=2)),
]


def frame(w, h, seed, gray=False):
    rng = np.random.default_rng(seed)
    g = synth.texture(w, h, seed)
    if gray:
        return g
    rgb = synth.to_bgr(g)[..., ::-1].copy()
    rgb[..., 0] = np.clip(rgb[..., 0].astype(np.int32) + rng.integers(-40, 41, (h, w)), 0, 255)
    return rgb.astype(np.uint8)


def main():
    out = {}
    for i, (name, w, h, opt) in enumerate(CASES):
        img = frame(w, h, 900 + i, gray=name.startswith("gray"))
        buf = io.BytesIO()
        Image.fromarray(img).save(buf, "JPEG", **opt)
        data = np.frombuffer(buf.getvalue(), np.uint8)
        bgr = np.asarray(Image.open(io.BytesIO(buf.getvalue())).convert("RGB"))[..., ::-1]
        out[f"{name}_jpeg"] = data
        out[f"{name}_bgr"] = np.ascontiguousarray(bgr)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jpeg_fixtures.npz"), **out)


if __name__ == "__main__":
    main()
