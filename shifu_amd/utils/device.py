"""Device helpers.  The GPU path is HIP/ROCm only; the CPU path exists for tests and
tiny LOCAL-mode runs."""
from __future__ import annotations

import os

import torch


def is_gpu_available() -> bool:
    if os.environ.get("SHIFU_FORCE_CPU") == "1":
        return False
    return torch.cuda.is_available()


def default_device() -> torch.device:
    if is_gpu_available():
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        return torch.device("cuda", lr % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def sync(device: torch.device | None = None) -> None:
    if device is None or device.type == "cuda":
        if torch.cuda.is_available():
            torch.cuda.synchronize()


def compute_dtype(device: torch.device) -> torch.dtype:
    """bf16 on MI355X (MFMA), fp32 on the CPU test path."""
    return torch.bfloat16 if device.type == "cuda" else torch.float32


def free_hbm(device) -> int:
    """Bytes of HBM this process can still allocate on ``device``: the driver's free memory plus
    the blocks the caching allocator holds but no tensor uses (a step that ran earlier in the same
    process -- e.g. the stats device cache before varsel in one pipeline -- leaves them reserved;
    the allocator releases them and retries when a new allocation does not fit).  Sizing decisions
    (resident vs streamed rows, cache budgets) use this, not ``mem_get_info`` alone."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return 0
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev))
