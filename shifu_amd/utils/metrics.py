"""Machine-readable JSONL metrics stream (rank 0 only).

Replaces the reference's HDFS progress-log side channel that the client tails every
2 s (``J/core/dtrain/nn/NNOutput.java:219-237``,
``J/core/processor/TrainModelProcessor.java:1862-1966``).
"""
from __future__ import annotations

import json
import os
import time


class MetricsWriter:
    def __init__(self, path: str | None, enabled: bool = True):
        self.path = path
        self.enabled = enabled and path is not None
        self._fh = None
        if self.enabled:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def write(self, **kv):
        if not self.enabled:
            return
        kv.setdefault("ts", time.time())
        self._fh.write(json.dumps(kv, default=float) + "\n")

    def write_raw(self, text: str):
        """Append already-serialised JSONL lines (another rank's stream)."""
        if self.enabled and text:
            self._fh.write(text if text.endswith("\n") else text + "\n")

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
