"""Process-group runtime: one process per GPU, RCCL over xGMI.

Replaces Guagua's BSP master/worker star (``J/core/processor/TrainModelProcessor.java:720-945``,
worker→master ``NNParams.doWrite`` ``J/core/dtrain/nn/NNParams.java:155-174``, master→worker
broadcast ``J/core/dtrain/nn/NNMaster.java:299-318``) with an all-reduce + replicated
optimizer: every rank holds the full (tiny) model and optimizer state, so the only
per-iteration traffic is one ``all_reduce(SUM)`` of the flat fp32 gradient buffer with the
error scalars fused into its tail.

On ROCm ``backend="nccl"`` *is* RCCL.  The CPU path uses ``gloo`` (tests / LOCAL mode).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as tdist

from ..utils.log import get_logger

_log = get_logger("parallel.dist")

# xGMI: 7 links x ~153 GB/s per MI355X.  RCCL stripes channels over links; a bucket needs
# >= ~1 MB per channel to engage them all, so default buckets are 16 MB.
DEFAULT_BUCKET_BYTES = 16 << 20


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_dist(self) -> bool:
        return self.world_size > 1

    @property
    def is_master(self) -> bool:
        return self.rank == 0


_INFO = DistInfo()
_LOCAL = 0      # > 0 inside local_only(): this rank runs a step alone, collectives are no-ops


def info() -> DistInfo:
    if _LOCAL:
        return DistInfo(0, 1, _INFO.local_rank, _INFO.backend)
    return _INFO


class local_only:
    """Run a block on this rank alone (the other ranks skip it): ``info()`` reports a world of
    one and barrier / all_reduce / broadcast / all_gather do nothing, so a step that is not
    data-parallel can run on rank 0 while the group waits at the next real collective."""

    def __enter__(self):
        global _LOCAL
        _LOCAL += 1
        return self

    def __exit__(self, *exc):
        global _LOCAL
        _LOCAL -= 1
        return False


def _active() -> bool:
    return not _LOCAL and tdist.is_initialized() and tdist.get_world_size() > 1


def init_from_env(backend: str | None = None, timeout_s: int = 1800) -> DistInfo:
    """Initialise from torchrun-style env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    global _INFO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and os.environ.get("SHIFU_FORCE_CPU") != "1"
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1 and not tdist.is_initialized():
        # SHIFU_DIST_BACKEND=gloo: host-transport collectives on a GPU box (tests of the device
        # contract with several ranks on one GPU; RCCL refuses two ranks per device)
        be = backend or os.environ.get("SHIFU_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if be == "nccl" and use_gpu:
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        tdist.init_process_group(backend=be, rank=rank, world_size=world,
                                 timeout=datetime.timedelta(seconds=timeout_s), **kw)
        _INFO = DistInfo(rank, world, local, be)
        _log.info("process group up: rank %d/%d backend=%s", rank, world, be)
    elif tdist.is_initialized():
        _INFO = DistInfo(tdist.get_rank(), tdist.get_world_size(), local, tdist.get_backend())
    else:
        _INFO = DistInfo(0, 1, local, "none")
    return _INFO


def set_info(i: DistInfo) -> None:
    global _INFO
    _INFO = i


def shutdown() -> None:
    if tdist.is_initialized():
        tdist.destroy_process_group()


def coll_device() -> torch.device:
    """Device a collective's tensors must live on: the rank's GPU under RCCL (``nccl`` cannot
    reduce host tensors), the host under gloo -- except under SHIFU_ASSERT_DEVICE_COLLECTIVES=1 on
    a GPU box, where gloo runs follow RCCL's contract so the guard sees the RCCL device choices."""
    if tdist.is_initialized() and (tdist.get_backend() == "nccl" or (
            os.environ.get("SHIFU_ASSERT_DEVICE_COLLECTIVES") == "1" and _compute_device_type() == "cuda")):
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _compute_device_type() -> str:
    return "cuda" if torch.cuda.is_available() and os.environ.get("SHIFU_FORCE_CPU") != "1" else "cpu"


def _stage_device() -> torch.device:
    """Where host values are staged for a collective (see coll_device)."""
    return coll_device()


def _check(t: torch.Tensor, what: str) -> None:
    """SHIFU_ASSERT_DEVICE_COLLECTIVES=1: every tensor handed to a collective must be on the
    device RCCL would need (the rank's GPU whenever there is one), whatever the backend -- so a
    gloo run on a GPU box (or a CPU run) catches a host tensor that would make RCCL raise."""
    if os.environ.get("SHIFU_ASSERT_DEVICE_COLLECTIVES") != "1":
        return
    want = _compute_device_type()
    if t.device.type != want:
        raise AssertionError(f"{what}: collective over a {t.device.type} tensor (rank compute device: {want})")


def barrier() -> None:
    if _active():
        if tdist.get_backend() == "nccl":
            tdist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            tdist.barrier()


def all_reduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if not _active():
        return t
    _check(t, "all_reduce")
    rop = {"sum": tdist.ReduceOp.SUM, "max": tdist.ReduceOp.MAX, "min": tdist.ReduceOp.MIN}[op]
    tdist.all_reduce(t, op=rop)
    return t


def all_reduce_np(a, op: str = "sum"):
    """All-reduce a host (numpy) array, staged through HBM when the backend is RCCL."""
    if not _active():
        return a
    import numpy as np
    t = torch.from_numpy(np.ascontiguousarray(a)).to(_stage_device())
    all_reduce_(t, op)
    return t.cpu().numpy()


def all_gather_objects(obj) -> list:
    """Every rank's (picklable, small) ``obj``, in rank order."""
    if not _active():
        return [obj]
    out = [None] * tdist.get_world_size()
    tdist.all_gather_object(out, obj)
    return out


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _active():
        _check(t, "broadcast")
        tdist.broadcast(t, src=src)
    return t


def all_gather_cat(t: torch.Tensor) -> torch.Tensor:
    """Gather variable-length 1-D tensors from all ranks and concatenate (rank order)."""
    if not _active():
        return t
    _check(t, "all_gather_cat")
    n = torch.tensor([t.numel()], device=t.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(tdist.get_world_size())]
    tdist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t.reshape(-1)
    outs = [torch.zeros_like(pad) for _ in sizes]
    tdist.all_gather(outs, pad)
    return torch.cat([o[: int(s.item())] for o, s in zip(outs, sizes)])


def gather_cat(t: torch.Tensor, dst: int = 0):
    """Concatenate every rank's variable-length 1-D ``t`` on rank ``dst`` (rank order); None on
    the others (a tensor gather - no pickling, and only ``dst`` holds the full array)."""
    if not _active():
        return t
    _check(t, "gather_cat")
    n = torch.tensor([t.numel()], device=t.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(tdist.get_world_size())]
    tdist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t.reshape(-1)
    r = tdist.get_rank()
    outs = [torch.zeros_like(pad) for _ in sizes] if r == dst else None
    tdist.gather(pad, outs, dst=dst)
    if r != dst:
        return None
    return torch.cat([o[: int(s.item())] for o, s in zip(outs, sizes)])


def row_block(n: int, rank: int | None = None, world: int | None = None) -> tuple:
    """[a, b) of ``n`` rows owned by ``rank`` in a block partition (blocks differ by <= 1 row)."""
    i = info()
    r = i.rank if rank is None else rank
    w = i.world_size if world is None else world
    q, m = divmod(n, w)
    a = r * q + min(r, m)
    return a, a + q + (1 if r < m else 0)


def reduce_scatter_rows(t: torch.Tensor, dim0: bool = False) -> torch.Tensor:
    """Sum ``t`` over ranks and return this rank's row block (``row_block`` of F).

    ``t`` is [K, F, C] (block [K, b - a, C]) or, with ``dim0``, [F, K, C] (block [b - a, K, C]):
    there a rank's rows are one contiguous slab, so when R divides F the tensor goes to RCCL's
    ``reduce_scatter_tensor`` as it is (no padded rank-major copy; each rank receives 1/R of the
    bytes an all-reduce would leave everywhere).  gloo (no reduce-scatter): all-reduce + slice."""
    if not _active():
        return t
    _check(t, "reduce_scatter_rows")
    w, r = tdist.get_world_size(), tdist.get_rank()
    F = t.shape[1] if not dim0 else t.shape[0]
    a, b = row_block(F, r, w)
    if tdist.get_backend() != "nccl":
        all_reduce_(t)
        return (t[a:b] if dim0 else t[:, a:b]).contiguous()
    fb = -(-F // w)
    if dim0 and F % w == 0:
        t = t.contiguous()
        out = torch.empty((fb,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        tdist.reduce_scatter_tensor(out.reshape(-1), t.reshape(-1), op=tdist.ReduceOp.SUM)
        return out
    if dim0:
        src = torch.zeros((w, fb) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        for k in range(w):
            ka, kb = row_block(F, k, w)
            src[k, : kb - ka] = t[ka:kb]
        out = torch.empty((fb,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        tdist.reduce_scatter_tensor(out.reshape(-1), src.reshape(-1), op=tdist.ReduceOp.SUM)
        return out[: b - a].contiguous()
    K, _, C = t.shape
    src = torch.zeros(w, K, fb, C, dtype=t.dtype, device=t.device)
    for k in range(w):
        ka, kb = row_block(F, k, w)
        src[k, :, : kb - ka] = t[:, ka:kb]
    out = torch.empty(K, fb, C, dtype=t.dtype, device=t.device)
    tdist.reduce_scatter_tensor(out.reshape(-1), src.reshape(-1), op=tdist.ReduceOp.SUM)
    return out[:, : b - a].contiguous()


def gather_rows_to(t: torch.Tensor, n: int, dst: int = 0):
    """Concatenate every rank's row block ``t`` [b - a, C] of an [n, C] matrix on rank ``dst``
    (None elsewhere)."""
    if not _active():
        return t
    _check(t, "gather_rows_to")
    w, r = tdist.get_world_size(), tdist.get_rank()
    fb = -(-n // w)
    pad = torch.zeros(fb, t.shape[1], dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.zeros_like(pad) for _ in range(w)] if r == dst else None
    tdist.gather(pad, outs, dst=dst)
    if r != dst:
        return None
    return torch.cat([outs[k][: row_block(n, k, w)[1] - row_block(n, k, w)[0]] for k in range(w)])


def all_reduce_max_scalar(x: float, device=None) -> float:
    """Max of a host scalar over ranks (staged on the collective device: RCCL needs HBM)."""
    if not _active():
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device if device is not None else _stage_device())
    all_reduce_(t, "max")
    return float(t.item())


class BucketedAllReducer:
    """All-reduce a flat buffer in fixed-size buckets, asynchronously.

    ``launch(upto)`` may be called repeatedly while a backward produces gradients
    back-to-front, so communication of finished buckets overlaps the remaining compute
    (HIP stream of the process group runs beside the compute stream).  ``wait()`` joins.
    """

    def __init__(self, flat: torch.Tensor, bucket_bytes: int = DEFAULT_BUCKET_BYTES):
        assert flat.dim() == 1
        self.flat = flat
        per = max(1, bucket_bytes // flat.element_size())
        self.bounds = [(i, min(i + per, flat.numel())) for i in range(0, flat.numel(), per)]
        self._handles = []
        self._launched = 0

    def reset(self):
        self._handles = []
        self._launched = 0

    def launch_all(self):
        self.launch_from(0)

    def launch_from(self, start_elem: int):
        """Launch every not-yet-launched bucket whose range lies entirely at >= start_elem
        (buckets are launched from the END of the buffer, matching a back-to-front backward)."""
        if not _active():
            return
        for bi in range(len(self.bounds) - 1 - self._launched, -1, -1):
            lo, hi = self.bounds[bi]
            if lo < start_elem:
                break
            _check(self.flat, "bucketed all_reduce")
            h = tdist.all_reduce(self.flat[lo:hi], op=tdist.ReduceOp.SUM, async_op=True)
            self._handles.append(h)
            self._launched += 1

    def wait(self):
        if not _active():
            return
        if self._launched < len(self.bounds):
            self.launch_from(0)
        for h in self._handles:
            h.wait()
        self.reset()
