"""Camera-per-rank sharding and the per-frame tracklet-slot all-gather.

The reference runs every camera's CPSNWhere_Tracker2D in one process and hands
the per-camera std::vector<stTrack2DResult> to CPSNWhere_Associator3D::Run
(psn_where/PSNWhere.cpp:253-269), which requires result2D[cam].camID == cam
(PSNWhere_Associator3D.cpp:1105-1116). Here one rank (one GPU) owns one camera
(rank == camera index) and the only exchange is one all-gather per frame of a
fixed-size slot per camera, so the gathered rows are ordered by camera index.

Slot layout (bytes, all offsets 4-byte aligned):
  [0, 16)            int32 header: cam, frame, npts, reserved
  [16, 16+8N)        float32 next_xy (LK output, written in place by the kernel)
  [16+8N, 16+12N)    float32 err
  [16+12N, 16+13N)   uint8 status
padded to a multiple of 64 bytes.

Works with any torch.distributed backend: nccl (= RCCL over xGMI on ROCm) for
device tensors, gloo for the CPU tests.
"""
from __future__ import annotations

HEADER_BYTES = 16


def slot_bytes(npts: int) -> int:
    n = HEADER_BYTES + 13 * npts
    return (n + 63) // 64 * 64


def slot_views(slot, npts: int):
    """(header int32[4], next_xy float32[npts,2], err float32[npts], status uint8[npts]) views of a
    uint8 torch tensor of slot_bytes(npts) bytes."""
    import torch

    assert slot.dtype == torch.uint8 and slot.numel() >= slot_bytes(npts)
    o = HEADER_BYTES
    header = slot[0:o].view(torch.int32)
    nxt = slot[o:o + 8 * npts].view(torch.float32).view(npts, 2)
    err = slot[o + 8 * npts:o + 12 * npts].view(torch.float32)
    status = slot[o + 12 * npts:o + 13 * npts]
    return header, nxt, err, status


def allgather_slots(slot, world_size: int, out=None):
    """All-gather one slot per rank -> tensor [world_size, slot_bytes], row r = camera r."""
    import torch
    import torch.distributed as dist

    if out is None:
        out = torch.empty((world_size, slot.numel()), dtype=slot.dtype, device=slot.device)
    if world_size == 1:
        out[0].copy_(slot)
        return out
    dist.all_gather_into_tensor(out.view(-1), slot)
    return out


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over all ranks (the bench's max-over-ranks timing)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
