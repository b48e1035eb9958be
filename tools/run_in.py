"""Run one shifu CLI verb inside a model-set directory (a profiler-friendly entry point: the
program after ``rocprofv3 --`` must be python itself, not a shell).

    python tools/run_in.py <model set dir> <verb> [args...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


if __name__ == "__main__":
    os.chdir(sys.argv[1])
    from shifu_amd.cli import main
    sys.exit(main(sys.argv[2:]))
