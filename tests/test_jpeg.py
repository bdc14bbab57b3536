"""JPEG frame ingest: cv::imread(..., IMREAD_COLOR) of every
camera's frame (psn_where/main.cpp:144) before CPSNWhere_Tracker2D::Run's
cvtColor(BGR2GRAY) (PSNWhere_Tracker2D.cpp:256-263), decoded on the device
(include/psn_jpeg.h).

Pinning: tests/golden/jpeg_fixtures.npz holds JPEG files encoded by PIL
(libjpeg-turbo) and PIL's own decodes (tests/golden/make_jpeg_golden.py); the
CPU restatement oracle/jpeg_oracle.c must equal them bit for bit, and the
device decoder must equal both. Parity with OpenCV 2.4.6's bundled libjpeg 8
for subsampled chroma is unpinned (see oracle/jpeg_oracle.c).
"""
import io
import os

import numpy as np
import pytest

from mcmtt_opticalflow_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jpeg_fixtures.npz")


def fixtures():
    z = np.load(GOLDEN)
    names = sorted({k[:-5] for k in z.files if k.endswith("_jpeg")})
    return [(n, z[n + "_jpeg"].tobytes(), z[n + "_bgr"]) for n in names]


def _pil_jpeg(img, **opt):
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", **opt)
    data = b.getvalue()
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))[..., ::-1]
    return data, np.ascontiguousarray(ref)


def _color_frame(sc, t):
    rgb = synth.to_bgr(sc.frame(t))[..., ::-1].copy()
    rgb[..., 0] = np.clip(rgb[..., 0].astype(np.int32) + ((np.arange(sc.width) * 7) % 61 - 30)[None, :], 0, 255)
    return rgb.astype(np.uint8)


# ------------------------------------------------------------------ CPU: oracle

def test_oracle_matches_fixtures(oracle_mod):
    for name, data, bgr in fixtures():
        np.testing.assert_array_equal(oracle_mod.jpeg_decode_bgr(data), bgr, err_msg=name)


@pytest.mark.parametrize("opt", [dict(quality=85, subsampling=2, restart_marker_rows=1),
                                 dict(quality=70, subsampling=2), dict(quality=92, subsampling=0)])
def test_oracle_matches_pil_1080p(oracle_mod, opt):
    pytest.importorskip("PIL")
    sc = synth.make_scene(5, 1920, 1080, 64)
    data, ref = _pil_jpeg(_color_frame(sc, 0), **opt)
    np.testing.assert_array_equal(oracle_mod.jpeg_decode_bgr(data), ref)


def test_jpeg_info_and_rejects():
    from mcmtt_opticalflow_amd import lk

    name, data, bgr = fixtures()[0]
    assert lk.JpegDecoder.info(data)[:2] == (bgr.shape[1], bgr.shape[0])
    with pytest.raises(Exception):
        lk.JpegDecoder.info(b"\x00\x01not a jpeg")
    pytest.importorskip("PIL")
    prog, _ = _pil_jpeg(np.zeros((16, 16, 3), np.uint8) + 100, quality=80, progressive=True)
    with pytest.raises(Exception):  # progressive is not the baseline path
        lk.JpegDecoder.info(prog)


def _with_dht(data: bytes, tc_th: int, bits, vals, before_sos: bool = False) -> bytes:
    """data with one more DHT segment: right after SOI (parsed before the file's
    own tables, which redefine its slot) or right before SOS (after them: the
    scan uses it)."""
    body = bytes([tc_th]) + bytes(bits) + bytes(vals)
    seg = b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body
    at = data.find(b"\xff\xda") if before_sos else 2
    return data[:at] + seg + data[at:]


_BAD_TABLES = {
    "two_1bit_codes": (0x00, [2] + [0] * 15, [0, 1]),
    "overfull_1bit": (0x00, [200] + [0] * 15, [0] * 200),  # the advisor's bits[0] = 200
    "all_ones_3bit": (0x10, [0, 0, 8] + [0] * 13, list(range(8))),
    "dc_symbol_200": (0x01, [0, 1] + [0] * 14, [200]),
    "ac_overflow": (0x11, [0, 3, 3] + [0] * 13, [1, 2, 3, 4, 5, 6]),
}


@pytest.mark.parametrize("case", sorted(_BAD_TABLES))
def test_jpeg_rejects_bad_huffman_tables(oracle_mod, case):
    """jdhuff.c jpeg_make_d_derived_tbl's JERR_BAD_HUFF_TABLE cases: a canonical
    code that overflows its length (would index past the 9-bit lookahead table),
    and DC symbols above 15 (shifts of >= 16 bits in extend). libjpeg checks the
    tables a scan uses, when the scan starts: a bad table the scan uses is
    refused by the device decoder's parser and the oracle (PSN_LK_ERR_ARG); the
    same table redefined by the file's own DHT before the scan, or put in a slot
    no component uses, is accepted and the frame decodes as before."""
    from mcmtt_opticalflow_amd import lk

    _, data, bgr = fixtures()[0]
    tc_th, bits, vals = _BAD_TABLES[case]
    used = _with_dht(data, tc_th, bits, vals, before_sos=True)
    with pytest.raises(lk.PsnLkError) as e:
        lk.JpegDecoder.info(used)
    assert e.value.code == -1  # PSN_LK_ERR_ARG
    with pytest.raises(ValueError):
        oracle_mod.jpeg_decode_bgr(used)
    for ok in (_with_dht(data, tc_th, bits, vals),  # redefined by the file's own table
               _with_dht(data, (tc_th & 0xF0) | 3, bits, vals, before_sos=True)):  # slot 3: unused
        assert lk.JpegDecoder.info(ok)[:2] == lk.JpegDecoder.info(data)[:2]
        np.testing.assert_array_equal(oracle_mod.jpeg_decode_bgr(ok), bgr)
    # a valid extra table (the JPEG standard's luminance DC table) is accepted
    ok = _with_dht(data, 0x03, [0, 1, 5, 1, 1, 1, 1, 1, 1] + [0] * 7, list(range(12)))
    assert lk.JpegDecoder.info(ok)[:2] == lk.JpegDecoder.info(data)[:2]


def test_jpeg_rejects_440_sampling():
    """4:4:0 (luma h1v2) has no upsampling path: refused as unsupported, never
    decoded with the h2v2 rule."""
    from mcmtt_opticalflow_amd import lk

    pytest.importorskip("PIL")
    data, _ = _pil_jpeg(np.zeros((32, 32, 3), np.uint8) + 90, quality=90, subsampling=0)
    b = bytearray(data)
    sof = b.find(b"\xff\xc0")
    assert sof > 0 and b[sof + 11] == 0x11  # component 0's sampling byte (h=1, v=1)
    b[sof + 11] = 0x12
    with pytest.raises(lk.PsnLkError) as e:
        lk.JpegDecoder.info(bytes(b))
    assert e.value.code == -8  # PSN_LK_ERR_UNSUPPORTED


# ------------------------------------------------------------------ GPU: device decoder

@pytest.mark.gpu
def test_device_decode_matches_fixtures():
    from mcmtt_opticalflow_amd import lk

    with lk.JpegDecoder() as dec:
        for name, data, bgr in fixtures():
            np.testing.assert_array_equal(dec.decode(data), bgr, err_msg=name)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [dict(quality=85, subsampling=2, restart_marker_rows=1),
                                 dict(quality=75, subsampling=2, restart_marker_blocks=4),
                                 dict(quality=70, subsampling=2), dict(quality=92, subsampling=0),
                                 dict(quality=60, subsampling=1, restart_marker_blocks=16)])
def test_device_decode_1080p(oracle_mod, opt):
    from mcmtt_opticalflow_amd import lk

    pytest.importorskip("PIL")
    sc = synth.make_scene(6, 1920, 1080, 64)
    data, ref = _pil_jpeg(_color_frame(sc, 1), **opt)
    with lk.JpegDecoder() as dec:
        got = dec.decode(data)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got, oracle_mod.jpeg_decode_bgr(data))


@pytest.mark.gpu
def test_push_frame_jpeg_pyramid(oracle_mod):
    """JPEG -> BGR -> cvtColor(BGR2GRAY) -> pyramid, all on the device, equals the
    oracle chain (decode, bgr2gray, buildOpticalFlowPyramid)."""
    from mcmtt_opticalflow_amd import lk

    pytest.importorskip("PIL")
    sc = synth.make_scene(7, 640, 480, 32)
    data, _ = _pil_jpeg(_color_frame(sc, 0), quality=88, subsampling=2, restart_marker_blocks=8)
    gray = oracle_mod.bgr2gray(oracle_mod.jpeg_decode_bgr(data))
    ref = oracle_mod.build_pyramid(gray, 4)
    with lk.LKContext(640, 480, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame_jpeg(1, data)
        ctx.sync()
        for lvl in range(4):
            np.testing.assert_array_equal(ctx.read_level(1, lvl), ref[lvl], err_msg=f"level {lvl}")


@pytest.mark.gpu
def test_group_run_from_jpeg_frames(oracle_mod):
    """Tracker2D Run fed with JPEG files gives the results of the same run fed
    with the decoded BGR frames (the decode is the only difference)."""
    from mcmtt_opticalflow_amd import tracker2d as t2d

    pytest.importorskip("PIL")
    W, H, C, T = 640, 480, 2, 4
    scenes = [synth.make_scene(70 + c, W, H, 96, nboxes=3, box_w=32, box_h=80) for c in range(C)]
    files = [[_pil_jpeg(_color_frame(sc, t), quality=90, subsampling=2, restart_marker_rows=1)[0]
              for t in range(T)] for sc in scenes]
    decoded = [[oracle_mod.jpeg_decode_bgr(f) for f in fs] for fs in files]

    def run(use_jpeg):
        out = []
        with t2d.Group(W, H, list(range(C)), max_objects=8) as g:
            for t in range(T):
                for c in range(C):
                    if use_jpeg:
                        g.push_frame_jpeg(c, files[c][t])
                    else:
                        g.push_frame(c, decoded[c][t])
                dets = []
                for sc in scenes:
                    pts = sc.points_at(t)
                    dets.append([t2d.make_detection((float(int(x)), float(int(y)), 32.0, 80.0), pts[sc.pt_box == k])
                                 for k, (x, y) in enumerate(sc.box_at(t))])
                out.append([r for _, r in g.run(t, dets)])
        return out

    a, b = run(True), run(False)
    n = 0
    for fa, fb in zip(a, b):
        for ra, rb in zip(fa, fb):
            assert len(ra["objects"]) == len(rb["objects"])
            for oa, ob in zip(ra["objects"], rb["objects"]):
                assert (oa["id"], oa["box"]) == (ob["id"], ob["box"])
                np.testing.assert_array_equal(oa["curr"], ob["curr"])
                n += 1
    assert n > 10
