"""Camera-per-rank sharding and the per-frame tracklet-slot all-gather.

The reference runs every camera's CPSNWhere_Tracker2D in one process and hands
the per-camera std::vector<stTrack2DResult> to CPSNWhere_Associator3D::Run
(psn_where/PSNWhere.cpp:253-269), which requires result2D[cam].camID == cam
(PSNWhere_Associator3D.cpp:1105-1116). Here one rank (one GPU) owns one camera
(rank == camera index) and the only exchange is one all-gather per frame of a
fixed-size slot per camera, so the gathered rows are ordered by camera index.

Slot layout of a rank holding C cameras of N points each (M = C*N points;
bytes, all offsets 4-byte aligned; C = 1 is the one-camera-per-GPU case):
  [0, 16C)             int32 header per camera: cam, frame, npts, reserved
  [16C, 16C+8M)        float32 next_xy, camera-major (LK output, written in place)
  [16C+8M, 16C+12M)    float32 err
  [16C+12M, 16C+13M)   uint8 status
padded to a multiple of 64 bytes.

Works with any torch.distributed backend: nccl (= RCCL over xGMI on ROCm) for
device tensors, gloo for the CPU tests.
"""
from __future__ import annotations

HEADER_BYTES = 16


def slot_bytes(npts: int, ncam: int = 1) -> int:
    """Bytes of one rank's slot: `ncam` cameras of `npts` points each."""
    n = HEADER_BYTES * ncam + 13 * npts * ncam
    return (n + 63) // 64 * 64


def slot_views(slot, npts: int, ncam: int = 1):
    """(header int32[4] (ncam == 1) or [ncam, 4], next_xy float32[M,2], err float32[M],
    status uint8[M]) views of a uint8 torch tensor of slot_bytes(npts, ncam) bytes, M = ncam*npts."""
    import torch

    assert slot.dtype == torch.uint8 and slot.numel() >= slot_bytes(npts, ncam)
    o = HEADER_BYTES * ncam
    header = slot[0:o].view(torch.int32)
    if ncam > 1:
        header = header.view(ncam, 4)
    npts = npts * ncam
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


def slot_offsets(npts: int, ncam: int = 1):
    """Byte offsets of (header, next_xy, err, status) in a slot of
    slot_bytes(npts, ncam) bytes (device pointers = slot base + offset)."""
    m = npts * ncam
    o = HEADER_BYTES * ncam
    return 0, o, o + 8 * m, o + 12 * m


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over all ranks (the bench's max-over-ranks timing; CPU
    tensors on the gloo control plane unless `device` names another)."""
    import sys

    if "torch.distributed" not in sys.modules:  # no control plane in this process: one rank
        return float(value)
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def init_comm(world: int, rank: int, device: int):
    """The library's RCCL communicator over all ranks (psn_comm_init); the unique
    id travels over the torch.distributed control group (gloo) when world > 1."""
    import ctypes

    from . import _lib

    L = _lib.load()
    uid = (ctypes.c_uint8 * _lib.COMM_UNIQUE_ID_BYTES)()
    if rank == 0 and L.psn_comm_get_unique_id(uid) != 0:
        raise RuntimeError("psn_comm_get_unique_id failed")
    if world > 1:
        import torch.distributed as dist

        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0)
        ctypes.memmove(uid, box[0], len(box[0]))
    comm = ctypes.c_void_p()
    rc = L.psn_comm_init(world, rank, device, uid, ctypes.byref(comm))
    if rc != 0:
        raise RuntimeError(f"psn_comm_init failed ({rc})")
    return comm


def comm_allgather(comm, d_send: int, d_recv: int, nbytes: int, stream: int):
    """psn_comm_allgather of one slot per rank, device to device, enqueued on `stream`."""
    from . import _lib

    rc = _lib.load().psn_comm_allgather(comm, d_send, d_recv, nbytes, stream)
    if rc != 0:
        raise RuntimeError(f"psn_comm_allgather failed ({rc})")


def comm_destroy(comm):
    from . import _lib

    _lib.load().psn_comm_destroy(comm)


class ResultExchange:
    """Per-frame hand-off of every camera's packed stTrack2DResult slot
    (psn_t2d_pack_result) into Associator3D: each rank contributes its C
    cameras' slots (rank r holds cameras r*C .. r*C+C-1), every rank receives
    all of them in camera order (index == camID, PSNWhere_Associator3D.cpp:
    1105-1116) in host memory.

    Pipelined: start(send) copies the frame's slots into a staging ring entry
    and enqueues the exchange, returning a ticket at once; wait(ticket) blocks
    only when the gathered slots are consumed (the bench consumes frame t's at
    step t+1, while frame t+1 runs on the GPU), so the exchange is off the host's
    critical path between one frame's completion and the next frame's launch.
    The reference hands the vector over in-process and Associator3D runs right
    after (PSNWhere.cpp:257-269); here it runs one frame behind Tracker2D. Up to
    `depth` exchanges may be in flight; tickets are waited in start order.

    backend "psn_comm": the library's RCCL communicator (psn_comm_init /
    psn_comm_allgather over xGMI; the unique id travels over the
    torch.distributed control group when world > 1): staging pinned host ->
    device -> all-gather -> pinned host, enqueued on one HIP stream of the
    library's runtime (hip.py, no torch.cuda) with an event per ticket. backend
    "torch": the same exchange with torch.distributed on CPU tensors (gloo,
    async_op), for the CPU tests."""

    def __init__(self, world: int, rank: int, bytes_per_rank: int, device: int = 0, backend: str = "psn_comm",
                 depth: int = 3):
        self.world, self.rank, self.nbytes, self.backend, self.depth = world, rank, bytes_per_rank, backend, depth
        self._comm = None
        self._next = 0        # ring entry of the next start
        self._inflight = []   # ring entries started, not yet waited (start order)
        if backend == "torch":
            import torch

            self._send = [torch.empty(bytes_per_rank, dtype=torch.uint8) for _ in range(depth)]
            self._recv = [torch.empty(world * bytes_per_rank, dtype=torch.uint8) for _ in range(depth)]
            self._work = [None] * depth
            return
        from . import _lib, hip

        self._L = _lib.load()
        self._hip = hip
        comm = init_comm(world, rank, device)
        self._comm = comm
        hip.set_device(device)
        # the library's HIP runtime (mcmtt_opticalflow_amd/hip.py): pinned staging,
        # device buffers, one exchange stream, an event per ring entry
        self._stream = hip.Stream()
        self._pinned = hip.PinnedAllocator()
        self._send_h = [self._pinned((bytes_per_rank,)) for _ in range(depth)]
        self._recv_h = [self._pinned((world * bytes_per_rank,)) for _ in range(depth)]
        self._send = [hip.DeviceBuffer(bytes_per_rank) for _ in range(depth)]
        self._recv_d = [hip.DeviceBuffer(world * bytes_per_rank) for _ in range(depth)]
        self._done = [hip.Event() for _ in range(depth)]

    def start(self, send) -> int:
        """Enqueue the exchange of `send` (uint8, bytes_per_rank bytes; copied
        before return, so the caller may refill it) and return its ticket. A
        failed start leaves every ticket in flight intact."""
        import numpy as np

        if len(self._inflight) >= self.depth:
            raise RuntimeError(f"ResultExchange: {self.depth} exchanges in flight; wait for the oldest first")
        src = np.ascontiguousarray(send).reshape(-1)
        if src.dtype != np.uint8 or src.size != self.nbytes:
            raise ValueError(f"ResultExchange.start: {src.size} {src.dtype} values, expected {self.nbytes} uint8")
        # the in-flight entries are the run just before _next (waited in start
        # order), so with fewer than `depth` in flight entry _next is free
        i = self._next
        if self.backend == "torch":
            import torch
            import torch.distributed as dist

            self._send[i].copy_(torch.from_numpy(src))
            self._work[i] = dist.all_gather_into_tensor(self._recv[i], self._send[i], async_op=True)
        else:
            h = self._hip
            self._send_h[i][:] = src  # a few KB: the caller's buffer is free again
            h.memcpy_async(self._send[i].addr, self._send_h[i].ctypes.data, self.nbytes, h.H2D, self._stream)
            rc = self._L.psn_comm_allgather(self._comm, self._send[i].addr, self._recv_d[i].addr, self.nbytes,
                                            self._stream.handle)
            if rc != 0:
                raise RuntimeError(f"psn_comm_allgather failed ({rc})")
            h.memcpy_async(self._recv_h[i].ctypes.data, self._recv_d[i].addr, self.world * self.nbytes, h.D2H,
                           self._stream)
            self._done[i].record(self._stream)
        self._inflight.append(i)  # only once the exchange is enqueued
        self._next = (i + 1) % self.depth
        return i

    def wait(self, ticket: int):
        """The gathered slots of `ticket` (the oldest exchange in flight): uint8
        numpy array [world * bytes_per_rank] in camera order, valid until this
        ring entry is started again (`depth` starts later)."""
        if not self._inflight or self._inflight[0] != ticket:
            raise RuntimeError("ResultExchange.wait: tickets are waited in start order")
        self._inflight.pop(0)
        if self.backend == "torch":
            self._work[ticket].wait()
            self._work[ticket] = None
            return self._recv[ticket].numpy()
        self._done[ticket].synchronize()
        return self._recv_h[ticket]

    def pending(self) -> int:
        return len(self._inflight)

    def allgather(self, send):
        """Blocking exchange: start + wait (uint8 numpy array [world * bytes_per_rank])."""
        return self.wait(self.start(send))

    def close(self):
        while self._inflight:
            self.wait(self._inflight[0])
        if self._comm is not None:
            self._stream.synchronize()
            self._L.psn_comm_destroy(self._comm)
            self._comm = None
            for e in self._done:
                e.destroy()
            for b in self._send + self._recv_d:
                b.free()
            self._pinned.close()
            self._stream.destroy()
