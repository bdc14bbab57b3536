"""Deterministic synthetic multi-camera video for the Tracker2D LK path.

Follows BASELINE.md section 2 ("Inputs (deterministic)"): per camera c a
band-limited background texture (seed 1000+c), K moving textured boxes with
U[-4,4]^2 px/frame velocities (seed 2000+c) and N points placed inside the
boxes (seed 3000+c). Frame t is rendered analytically at the shifted phase
(not warped), so the true flow of every point is its box velocity.

The reference has no datasets in-tree (PETS2009 frames are read from disk at
psn_where/main.cpp:133-151), so every run here uses this synthetic video.
"""
from __future__ import annotations

import dataclasses

import numpy as np

NCOMP = 16


def _texture_params(seed: int, ncomp: int = NCOMP):
    rng = np.random.default_rng(seed)
    return dict(
        a=rng.uniform(4.0, 14.0, ncomp),
        wx=rng.uniform(0.05, 0.6, ncomp),
        wy=rng.uniform(0.05, 0.6, ncomp),
        px=rng.uniform(0.0, 2 * np.pi, ncomp),
        py=rng.uniform(0.0, 2 * np.pi, ncomp),
    )


def _render(params, xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
    """sum_k a_k sin(wx_k x + px_k) sin(wy_k y + py_k) on the grid ys x xs
    (separable: one outer product per component)."""
    sx = np.sin(np.outer(params["wx"], xs) + params["px"][:, None])  # (k, W)
    sy = np.sin(np.outer(params["wy"], ys) + params["py"][:, None])  # (k, H)
    return np.einsum("k,kh,kw->hw", params["a"], sy, sx, optimize=True)


def texture(width: int, height: int, seed: int) -> np.ndarray:
    """A static band-limited u8 texture (the scene background of camera `seed`)."""
    img = 128.0 + _render(_texture_params(1000 + seed), np.arange(width, dtype=np.float64),
                          np.arange(height, dtype=np.float64))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


@dataclasses.dataclass
class CameraScene:
    cam: int
    width: int
    height: int
    box_w: int              # uniform box size (the largest box under a size distribution)
    box_h: int
    boxes0: np.ndarray      # (K, 2) top-left at t=0
    vel: np.ndarray         # (K, 2) px/frame
    pts0: np.ndarray        # (N, 2) float32 at t=0
    pt_box: np.ndarray      # (N,) box index of each point
    bg: np.ndarray          # (H, W) float64 background intensity (before clamp)
    box_params: list
    box_ws: np.ndarray = None  # (K,) per-box width / height (int)
    box_hs: np.ndarray = None

    def __post_init__(self):
        k = len(self.boxes0)
        if self.box_ws is None:
            self.box_ws = np.full(k, self.box_w, np.int64)
        if self.box_hs is None:
            self.box_hs = np.full(k, self.box_h, np.int64)

    def box_size(self, k: int) -> tuple[int, int]:
        return int(self.box_ws[k]), int(self.box_hs[k])

    def box_at(self, t: float) -> np.ndarray:
        return self.boxes0 + self.vel * t

    def points_at(self, t: float) -> np.ndarray:
        return (self.pts0 + self.vel[self.pt_box] * t).astype(np.float32)

    def frame(self, t: int) -> np.ndarray:
        img = self.bg.copy()
        ys = np.arange(self.height, dtype=np.float64)
        xs = np.arange(self.width, dtype=np.float64)
        for k, (bx, by) in enumerate(self.box_at(t)):
            bw, bh = self.box_size(k)
            x0, x1 = int(np.ceil(bx)), int(np.ceil(bx + bw))
            y0, y1 = int(np.ceil(by)), int(np.ceil(by + bh))
            x0, y0 = max(x0, 0), max(y0, 0)
            x1, y1 = min(x1, self.width), min(y1, self.height)
            if x1 <= x0 or y1 <= y0:
                continue
            img[y0:y1, x0:x1] = 128.0 + _render(self.box_params[k], xs[x0:x1] - bx, ys[y0:y1] - by)
        return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def pets_box_sizes(cam: int, nboxes: int, height: int) -> tuple[np.ndarray, np.ndarray]:
    """Seeded PETS2009-like pedestrian boxes (seed 4000+cam): heights U[0.14,
    0.35] of the frame height (150..375 px at 1080p; PETS S2.L1 people span
    roughly 80..200 of its 576 rows), width/height U[0.35, 0.45] -- widths of
    any residue mod 8, as real detections have."""
    rng = np.random.default_rng(4000 + cam)
    hs = np.floor(rng.uniform(0.14, 0.35, nboxes) * height).astype(np.int64)
    ws = np.floor(hs * rng.uniform(0.35, 0.45, nboxes)).astype(np.int64)
    return np.maximum(ws, 8), np.maximum(hs, 8)


def make_scene(cam: int, width: int, height: int, npts: int, nboxes: int | None = None,
               box_w: int | None = None, box_h: int | None = None, max_speed: float = 4.0,
               box_dist: str = "uniform") -> CameraScene:
    """Box sizes per BASELINE.md: 32x80 at 640x480, 64x160 at 1080p, 128x320 at 4K
    (box_dist "uniform"), or per box from pets_box_sizes (box_dist "pets")."""
    if box_w is None:
        box_w = 32 if width <= 640 else 64 if width <= 1920 else 128
    if box_h is None:
        box_h = int(box_w * 2.5)
    if nboxes is None:
        nboxes = max(1, min(16, npts // 32))
    if box_dist == "pets":
        bws, bhs = pets_box_sizes(cam, nboxes, height)
        box_w, box_h = int(bws.max()), int(bhs.max())
    elif box_dist == "uniform":
        bws, bhs = np.full(nboxes, box_w, np.int64), np.full(nboxes, box_h, np.int64)
    else:
        raise ValueError(f"box_dist {box_dist!r}")
    bgp = _texture_params(1000 + cam)
    xs = np.arange(width, dtype=np.float64)
    ys = np.arange(height, dtype=np.float64)
    bg = 128.0 + _render(bgp, xs, ys)
    rng = np.random.default_rng(2000 + cam)
    mx = np.minimum(8 * max_speed + 8, np.maximum(0.0, (width - bws) / 2 - 1))
    my = np.minimum(8 * max_speed + 8, np.maximum(0.0, (height - bhs) / 2 - 1))
    boxes0 = np.stack([rng.uniform(mx, np.maximum(mx, width - bws - mx), nboxes),
                       rng.uniform(my, np.maximum(my, height - bhs - my), nboxes)], axis=1)
    vel = rng.uniform(-max_speed, max_speed, (nboxes, 2))
    box_params = [_texture_params(2000 + cam * 1000 + 17 * k + 1) for k in range(nboxes)]
    prng = np.random.default_rng(3000 + cam)
    pt_box = np.arange(npts) % nboxes
    inner = np.stack([prng.uniform(4, bws[pt_box] - 4, npts), prng.uniform(4, bhs[pt_box] - 4, npts)], axis=1)
    pts0 = (boxes0[pt_box] + inner).astype(np.float32)
    return CameraScene(cam, width, height, box_w, box_h, boxes0, vel, pts0, pt_box, bg, box_params, bws, bhs)


def to_bgr(gray: np.ndarray) -> np.ndarray:
    """A deterministic colour frame around the gray rendering (the reference
    ingests BGR frames from imread, main.cpp:144, and converts them with
    cvtColor(BGR2GRAY), PSNWhere_Tracker2D.cpp:257): G = gray, B = gray + 24,
    R = gray - 9 (clipped), chroma chosen so that the BT.601 luma of the colour
    frame is the gray frame (0.114 * 24 - 0.299 * 9 ~ 0): the tracked images
    keep the full contrast of the rendering."""
    g = gray.astype(np.int32)
    return np.stack([np.clip(g + 24, 0, 255), g, np.clip(g - 9, 0, 255)], axis=-1).astype(np.uint8)
