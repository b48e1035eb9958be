"""Command line (A1): ``shifu <command> [options]`` with ``-Dkey=value`` overrides.

Same verbs and single-dash options as ``ShifuCLI`` (J/ShifuCLI.java:145-428, option table
:702-813, usage :818-866).  ``train`` (and the other GPU-heavy verbs) run data-parallel when
launched under ``torchrun`` (``bin/shifu`` does that for ``SHIFU_GPUS>1``): each rank reads
RANK/LOCAL_RANK/WORLD_SIZE from the environment and joins the RCCL process group.
"""
from __future__ import annotations

import os
import time
import sys

from . import __version__
from .config import environment
from .utils.log import get_logger, setup_logging

USAGE = """Usage: shifu <command> [options]
  new <ModelSetName> [-t NN|LR|GBT|RF|WDL] [-m <description>]   create a model set
  init [-autotype] | init -model                               create ColumnConfig.json | fill default train params
  cp <src ModelSet> <dst ModelSet>                             copy a model set's ModelConfig.json
  stats [-c] [-p] [-rebin [-vars v1,v2] [-n <bins>] [-ivr <ratio>] [-bic <min count>]]
  norm|normalize|transform [-shuffle]                          normalize training data
  varsel|varselect [-reset|-list|-autofilter|-recoverauto] [-r <n>]  variable selection
  train [-dry] [-debug] [-shuffle]                             train models
  posttrain                                                    bin average scores / feature importance
  eval [-new <n>|-list|-delete <n>|-run [n]|-score [n] [-nosort]|-norm [n] [-strict]|-confmat [n]|-perf [n]]
  export -t pmml|columnstats|woemapping|bagging|baggingpmml|corr|woe [-c] [-vars v1,v2] [-n <bins>] [-ivr <ratio>] [-bic <cnt>]
  combo -new <algs>|-init|-run [-shuffle] [-resume]|-eval      stacking of sub models
  save [<name>] | switch <name> | show | list                  model-set branches
  encode [-run [<evalset>|*]] [-ref <modelset>]                tree leaf-path encoding
  test -filter [<evalset>|*] [-n <records>]                    dry-run filter expressions
  convert -tozipb|-totreeb <src> <dst>                         binary <-> readable tree models
  analysis -fi <model.gbt>                                     tree feature importance
  version | help
  -Dkey=value                                                  override a shifuconfig property"""

_log = get_logger("cli")

# verbs whose every rank takes part (row-sharded data, collectives inside); the other
# multi-GPU verbs run on rank 0 alone under dist.local_only()
DP_VERBS = ("train", "stats", "eval", "norm", "normalize", "transform", "varsel", "posttrain", "init",
            "encode", "combo")


def torch_status(rc: int):
    import torch
    from .parallel import dist as _d
    dev = _d.coll_device() if _d.info().world_size > 1 else "cpu"
    return torch.tensor([int(rc or 0)], dtype=torch.int64, device=dev)


def _opt(args, name, default=None, has_value=False):
    if name in args:
        i = args.index(name)
        if has_value:
            v = args[i + 1] if i + 1 < len(args) and not args[i + 1].startswith("-") else default
            return v
        return True
    return default


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    argv = environment.apply_cli_overrides(argv)
    setup_logging()
    if not argv or argv[0] in ("help", "-h", "--help"):
        print(USAGE)
        return 0
    cmd, args = argv[0].lower(), argv[1:]
    from .parallel import dist
    if cmd in DP_VERBS:
        dist.init_from_env()
    from .utils.trace import step_timer
    from .utils.telemetry import record_usage
    t0, rc = time.time(), 1
    try:
        with step_timer(cmd):
            info0 = dist.info()
            if info0.world_size > 1 and cmd not in DP_VERBS:
                # not data-parallel (yet): rank 0 runs the step alone, the others wait for it
                rc = 0
                if info0.rank == 0:
                    with dist.local_only():
                        rc = _dispatch(cmd, args)
                st = torch_status(rc)
                dist.all_reduce_(st, "max")
                rc = int(st.item())
                return rc
            rc = _dispatch(cmd, args)
            return rc
    except Exception as e:      # noqa: BLE001 - processors report errors and return non-zero
        if environment.get_bool("shifu.debug", False) or os.environ.get("SHIFU_DEBUG") == "1":
            raise
        _log.error("Error: %s: %s", type(e).__name__, e)
        return 1
    finally:
        info = dist.info()
        record_usage(cmd, args, rc if isinstance(rc, int) else 0, time.time() - t0, info.world_size, info.rank)
        if info.world_size > 1:
            dist.shutdown()


def _dispatch(cmd, args) -> int:
    if cmd in ("version", "-v", "--version"):
        print(f"shifu_amd {__version__}")
        return 0
    if cmd == "new":
        from .steps.create import run_new
        if not args:
            print(USAGE)
            return 1
        return run_new(args[0], _opt(args, "-t", "NN", True), _opt(args, "-m", None, True))
    if cmd == "cp":
        from .steps.create import copy_model_set
        rest = [a for a in args if not a.startswith("-")]
        if len(rest) < 2:
            print(USAGE)
            return 1
        return copy_model_set(rest[0], rest[1])
    if cmd == "init":
        from .steps.create import init_model_params, run_init
        if _opt(args, "-model"):
            return init_model_params(".")
        return run_init(".", True if _opt(args, "-autotype") else None)
    if cmd == "stats":
        from .steps.stats import run_stats
        n = _opt(args, "-n", None, True)
        ivr = _opt(args, "-ivr", None, True)
        bic = _opt(args, "-bic", None, True)
        vars_ = _opt(args, "-vars", None, True)
        return run_stats(".", bool(_opt(args, "-c") or _opt(args, "-correlation")),
                         bool(_opt(args, "-p") or _opt(args, "-psi")), bool(_opt(args, "-rebin")),
                         int(n) if n else None, float(ivr) if ivr else 1.0,
                         min_inst_cnt=float(bic) if bic else 0, request_vars=vars_.split(",") if vars_ else None)
    if cmd in ("norm", "normalize", "transform"):
        from .steps.norm import run_norm
        return run_norm(".", shuffle=bool(_opt(args, "-shuffle")))
    if cmd in ("varsel", "varselect"):
        from .steps.varsel import run_varsel
        r = _opt(args, "-r", None, True)
        return run_varsel(".", bool(_opt(args, "-reset")), bool(_opt(args, "-list")), bool(_opt(args, "-autofilter")),
                          bool(_opt(args, "-recoverauto")), int(r) if r else 1)
    if cmd == "train":
        from .steps.norm import run_norm
        from .steps.train import run_train
        if _opt(args, "-debug"):
            import logging
            logging.getLogger("shifu_amd").setLevel(logging.DEBUG)
        if _opt(args, "-shuffle"):
            run_norm(".", shuffle=True)
        return run_train(".", dry=bool(_opt(args, "-dry")))
    if cmd == "posttrain":
        from .steps.posttrain import run_posttrain
        return run_posttrain(".")
    if cmd == "eval":
        from .steps.evaluate import run_eval
        for a in ("new", "list", "delete", "run", "score", "norm", "confmat", "perf"):
            if f"-{a}" in args:
                return run_eval(".", a, _opt(args, f"-{a}", None, True), nosort=bool(_opt(args, "-nosort")),
                                strict=bool(_opt(args, "-strict")))
        return run_eval(".", "run", None)          # no option: every eval set
    if cmd == "export":
        from .steps.export import run_export
        vars_ = _opt(args, "-vars", None, True)
        n, ivr, bic = _opt(args, "-n", None, True), _opt(args, "-ivr", None, True), _opt(args, "-bic", None, True)
        return run_export(".", _opt(args, "-t", "pmml", True), bool(_opt(args, "-c")),
                          request_vars=vars_.split(",") if vars_ else None, expected_bins=int(n) if n else 0,
                          iv_keep_ratio=float(ivr) if ivr else 1.0, min_inst_cnt=float(bic) if bic else 0)
    if cmd == "combo":
        from .steps.combo import run_combo
        for a in ("new", "init", "run", "eval"):
            if f"-{a}" in args:
                return run_combo(".", a, _opt(args, "-new", None, True) if a == "new" else None,
                                 shuffle=bool(_opt(args, "-shuffle")), resume=bool(_opt(args, "-resume")))
        print(USAGE)
        return 1
    if cmd in ("save", "switch", "show", "list"):
        from .steps.misc import run_manage
        return run_manage(".", cmd, args[0] if args else None)
    if cmd == "encode":
        from .steps.misc import run_encode
        return run_encode(".", _opt(args, "-run", None, True), _opt(args, "-ref", None, True))
    if cmd == "test":
        from .steps.misc import run_filter_test
        n = _opt(args, "-n", None, True)
        return run_filter_test(".", _opt(args, "-filter", None, True), int(n) if n else 100)
    if cmd == "convert":
        from .steps.misc import run_convert
        mode = "tozipb" if "-tozipb" in args else "totreeb" if "-totreeb" in args else None
        rest = [a for a in args if not a.startswith("-")]
        if mode is None or len(rest) < 2:
            print(USAGE)
            return 1
        return run_convert(mode, rest[0], rest[1])
    if cmd == "analysis":
        from .steps.misc import run_analysis_fi
        m = _opt(args, "-fi", None, True)
        if not m:
            print(USAGE)
            return 1
        return run_analysis_fi(m)
    print(f"unknown command {cmd}\n{USAGE}")
    return 1


if __name__ == "__main__":
    sys.exit(main())
