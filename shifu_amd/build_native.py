"""Build the in-tree native libraries (no JIT cache: the .so files travel with the repo).

    python -m shifu_amd.build_native [--force] [-j N]

* every ``shifu_amd/ops/csrc/*.hip`` -> object with ``hipcc --offload-arch=gfx950`` ->
  ``shifu_amd/ops/_lib/libshifu_hip.so``
* every ``shifu_amd/runtime/csrc/*.cpp`` -> ``g++ -O3`` -> ``shifu_amd/ops/_lib/libshifu_rt.so``

Incremental on mtimes (headers count as dependencies of every source in their dir).
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
HIP_SRC = ROOT / "ops" / "csrc"
RT_SRC = ROOT / "runtime" / "csrc"
LIB_DIR = ROOT / "ops" / "_lib"
OBJ_DIR = LIB_DIR / "obj"
ARCH = os.environ.get("SHIFU_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found")


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1]}")
    return r


def build_hip(force=False, jobs=8, verbose=False) -> Path:
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sorted(HIP_SRC.glob("*.hip"))
    hdrs = sorted(HIP_SRC.glob("*.h"))
    hipcc = _hipcc()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", f"-I{HIP_SRC}"]
    objs, todo = [], []
    for s in srcs:
        o = OBJ_DIR / (s.stem + ".hip.o")
        objs.append(o)
        if force or _newer(o, [s, *hdrs]):
            todo.append([hipcc, *flags, "-c", str(s), "-o", str(o)])
    if todo:
        with ThreadPoolExecutor(max(1, jobs)) as ex:
            for r in ex.map(_run, todo):
                if verbose and r.stderr:
                    sys.stderr.write(r.stderr)
    out = LIB_DIR / "libshifu_hip.so"
    if force or todo or _newer(out, objs):
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out)])
    return out


def build_rt(force=False, jobs=8) -> Path | None:
    srcs = sorted(RT_SRC.glob("*.cpp"))
    if not srcs:
        return None
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hdrs = sorted(RT_SRC.glob("*.h"))
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-march=x86-64-v2", f"-I{RT_SRC}"]
    objs, todo = [], []
    for s in srcs:
        o = OBJ_DIR / (s.stem + ".cpp.o")
        objs.append(o)
        if force or _newer(o, [s, *hdrs]):
            todo.append([cxx, *flags, "-c", str(s), "-o", str(o)])
    if todo:
        with ThreadPoolExecutor(max(1, jobs)) as ex:
            list(ex.map(_run, todo))
    out = LIB_DIR / "libshifu_rt.so"
    if force or todo or _newer(out, objs):
        _run([cxx, "-shared", "-pthread", *map(str, objs), "-o", str(out), "-lz"])
    return out


def build_all(force=False, jobs=None, verbose=False):
    jobs = jobs or min(8, os.cpu_count() or 4)
    rt = build_rt(force, jobs)
    hip = build_hip(force, jobs, verbose)
    return hip, rt


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    hip, rt = build_all(a.force, a.j, a.v)
    print(f"built {hip}" + (f" and {rt}" if rt else ""))


if __name__ == "__main__":
    main()
