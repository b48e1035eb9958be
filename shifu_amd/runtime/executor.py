"""Local concurrency helpers (E6).

The reference's ``ExecutorManager`` (a thread pool whose failed tasks are re-submitted) and
``ProcessManager`` (runs ``shifu ...`` as child processes) drive combo sub-model training
(J/core/processor/ComboModelProcessor.java:278-356) and other fan-out work.  Here:

* ``ExecutorManager(workers, retries).run(tasks)`` - runs callables on a thread pool, re-runs a
  failed task up to ``retries`` times, raises the last error of a task that never succeeds;
* ``run_cli(args, cwd)`` - one ``shifu_amd.cli`` verb in a child process (its own GPU context,
  so sub-model pipelines can run side by side); returns the exit code;
* ``DevicePool`` - the node's GPUs as slots: a child process takes a free GPU for its whole task
  (``HIP_VISIBLE_DEVICES`` = that one device) and gives it back when done, so two children never
  share a device (each sizes its HBM caches to the whole card).
"""
from __future__ import annotations

import os
import queue
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from ..utils.log import get_logger

_log = get_logger("runtime.executor")


class TaskFailed(RuntimeError):
    pass


class ExecutorManager:
    def __init__(self, workers: int = 1, retries: int = 0):
        self.workers = max(1, int(workers))
        self.retries = max(0, int(retries))

    def _attempt(self, name, fn):
        err = None
        for attempt in range(self.retries + 1):
            try:
                return fn()
            except Exception as e:       # noqa: BLE001 - retried, then re-raised
                err = e
                _log.warning("task %s failed (attempt %d/%d): %s", name, attempt + 1, self.retries + 1, e)
        raise TaskFailed(f"task {name} failed after {self.retries + 1} attempts: {err}") from err

    def run(self, tasks, names=None):
        """Run ``tasks`` (callables); results in task order."""
        names = list(names) if names is not None else [str(i) for i in range(len(tasks))]
        if self.workers == 1 or len(tasks) <= 1:
            return [self._attempt(n, t) for n, t in zip(names, tasks)]
        with ThreadPoolExecutor(self.workers) as pool:
            futs = [pool.submit(self._attempt, n, t) for n, t in zip(names, tasks)]
            return [f.result() for f in futs]


class DevicePool:
    """GPU slots for child processes (one child per device at any time)."""

    def __init__(self, ids):
        self.ids = [str(i) for i in ids]
        self._free = queue.Queue()
        for i in self.ids:
            self._free.put(i)

    def __len__(self):
        return len(self.ids)

    @classmethod
    def for_node(cls):
        """This process's visible GPUs (``HIP_VISIBLE_DEVICES`` order), or None without a GPU.
        Counting devices does not initialise the GPU in this process."""
        if os.environ.get("SHIFU_FORCE_CPU") == "1":
            return None
        import torch
        n = torch.cuda.device_count()
        if n <= 0:
            return None
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
        ids = [v.strip() for v in vis.split(",") if v.strip()][:n] if vis else list(range(n))
        return cls(ids)

    def acquire(self) -> str:
        return self._free.get()

    def release(self, dev: str) -> None:
        self._free.put(dev)


def run_cli(args, cwd: str, env: dict | None = None, log_path: str | None = None) -> int:
    """``python -m shifu_amd.cli <args>`` in ``cwd`` as a child process -> exit code."""
    e = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    if env:
        e.update(env)
    out = open(log_path, "a") if log_path else subprocess.DEVNULL
    try:
        return subprocess.call([sys.executable, "-m", "shifu_amd.cli", *args], cwd=cwd, env=e,
                               stdout=out, stderr=subprocess.STDOUT)
    finally:
        if log_path:
            out.close()


def cli_task(steps, cwd: str, log_path: str | None = None, devices: DevicePool | None = None):
    """A callable running CLI verbs in order in child processes; raises on the first failure.
    ``devices``: the task holds one GPU of the pool for all its verbs (the children see only it)."""
    def run():
        dev = devices.acquire() if devices is not None else None
        env = None if dev is None else {"HIP_VISIBLE_DEVICES": dev, "LOCAL_RANK": "0"}
        try:
            for st in steps:
                args = st.split() if isinstance(st, str) else list(st)
                rc = run_cli(args, cwd, env=env, log_path=log_path)
                if rc != 0:
                    raise RuntimeError(f"'shifu {' '.join(args)}' in {cwd} exited with {rc}")
        finally:
            if dev is not None:
                devices.release(dev)
        return 0
    return run
