"""Local concurrency helpers (E6).

The reference's ``ExecutorManager`` (a thread pool whose failed tasks are re-submitted) and
``ProcessManager`` (runs ``shifu ...`` as child processes) drive combo sub-model training
(J/core/processor/ComboModelProcessor.java:278-356) and other fan-out work.  Here:

* ``ExecutorManager(workers, retries).run(tasks)`` - runs callables on a thread pool, re-runs a
  failed task up to ``retries`` times, raises the last error of a task that never succeeds;
* ``run_cli(args, cwd)`` - one ``shifu_amd.cli`` verb in a child process (its own GPU context,
  so sub-model pipelines can run side by side); returns the exit code.
"""
from __future__ import annotations

import os
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


def cli_task(steps, cwd: str, log_path: str | None = None):
    """A callable running CLI verbs in order in a child process; raises on the first failure."""
    def run():
        for st in steps:
            args = st.split() if isinstance(st, str) else list(st)
            rc = run_cli(args, cwd, log_path=log_path)
            if rc != 0:
                raise RuntimeError(f"'shifu {' '.join(args)}' in {cwd} exited with {rc}")
        return 0
    return run
