"""The product hand-off into Associator3D on the device: psn_comm (RCCL) on one
GPU. Every camera's stTrack2DResult from a psn_t2d_group Run is packed
(psn_t2d_pack_result), all-gathered with psn_comm_allgather (a one-rank
communicator: the same RCCL calls the multi-GPU bench makes per frame) and
unpacked bit for bit in camera order (index == camID,
PSNWhere_Associator3D.cpp:1105-1116; the in-process hand-off it replaces is
PSNWhere.cpp:257-269)."""
import ctypes

import numpy as np
import pytest

from mcmtt_opticalflow_amd import _lib, synth
from mcmtt_opticalflow_amd import tracker2d as t2d

pytestmark = pytest.mark.gpu


def test_psn_comm_allgather_packed_results_one_rank():
    import hiprt

    L, T = _lib.load(), t2d.load()
    W, H, C, F = 640, 480, 2, 4
    scenes = [synth.make_scene(60 + c, W, H, 96, nboxes=3, box_w=32, box_h=80) for c in range(C)]
    frames = [[synth.to_bgr(sc.frame(t)) for t in range(F)] for sc in scenes]
    slot = t2d.result_slot_bytes(8, 1)
    uid = (ctypes.c_uint8 * _lib.COMM_UNIQUE_ID_BYTES)()
    assert L.psn_comm_get_unique_id(uid) == 0
    comm = ctypes.c_void_p()
    assert L.psn_comm_init(1, 0, 0, uid, ctypes.byref(comm)) == 0
    n_obj = 0
    try:
        with t2d.Group(W, H, [0, 1], max_objects=8) as g:
            for t in range(F):
                for c in range(C):
                    g.push_frame(c, frames[c][t])
                dets = []
                for sc in scenes:
                    pts = sc.points_at(t)
                    dets.append([t2d.make_detection((float(int(x)), float(int(y)), 32.0, 80.0), pts[sc.pt_box == k])
                                 for k, (x, y) in enumerate(sc.box_at(t))])
                out = g.run(t, dets)
                send = np.zeros((C, slot), np.uint8)
                for c in range(C):
                    assert T.psn_t2d_pack_result(ctypes.byref(g.result_struct(c)), send[c].ctypes.data, slot) == 0
                d_send, d_recv = hiprt.DeviceBuffer.from_array(send), hiprt.DeviceBuffer(send.nbytes)
                assert L.psn_comm_allgather(comm, d_send.addr, d_recv.addr, send.nbytes, None) == 0
                recv = d_recv.to_array((C, slot), np.uint8)
                for c in range(C):
                    got, want = t2d.unpack_result(recv[c], 8, 1), out[c][1]
                    assert got["cam_id"] == c and got["frame_idx"] == t
                    assert len(got["objects"]) == len(want["objects"])
                    for a, b in zip(got["objects"], want["objects"]):
                        assert (a["id"], a["box"], a["head"], a["score"]) == (b["id"], b["box"], b["head"], b["score"])
                        np.testing.assert_array_equal(a["prev"], b["prev"])
                        np.testing.assert_array_equal(a["curr"], b["curr"])
                    n_obj += len(got["objects"])
    finally:
        L.psn_comm_destroy(comm)
    assert n_obj >= 2 * C * F
