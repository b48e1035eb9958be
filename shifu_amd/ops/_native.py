"""Loader for the in-tree native libraries.

* ``_lib/libshifu_hip.so`` - hand-written CDNA4 HIP kernels (built with
  ``hipcc --offload-arch=gfx950``; sources ``shifu_amd/ops/csrc/*.hip``).
* ``_lib/libshifu_rt.so``  - host C++ runtime (CSV parser, thread pool, binary IO;
  sources ``shifu_amd/runtime/csrc/*.cpp``).

Both are plain C ABIs loaded with :mod:`ctypes` so that device pointers / HIP streams are
passed straight from torch tensors with no Python<->C++ ABI coupling.  On a GPU box a
missing HIP library is a hard error (no silent eager fallback): callers on the GPU path use
:func:`hip` which raises :class:`NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "_lib"
# SHIFU_HIP_LIB: another build of the kernel library (same-box A/B runs of two builds in a lab)
HIP_LIB = Path(os.environ["SHIFU_HIP_LIB"]) if os.environ.get("SHIFU_HIP_LIB") else LIB_DIR / "libshifu_hip.so"
RT_LIB = LIB_DIR / "libshifu_rt.so"

_lock = threading.Lock()
_hip = None
_rt = None

# argument codes: p=void*, l=int64, i=int32, f=float, d=double, s=hipStream_t
_T = {"p": ctypes.c_void_p, "l": ctypes.c_long, "i": ctypes.c_int, "f": ctypes.c_float,
      "d": ctypes.c_double, "s": ctypes.c_void_p, "P": ctypes.c_char_p, "L": ctypes.c_long}

HIP_SIGNATURES = {
    # mlp_kernels.hip
    "shifu_gemm_nt": "plplipl" "plplpl" "iiiiiiif" "s",
    "shifu_wgrad_tn": "plplpl" "iiiis",
    "shifu_gemm_head": "plplipl" "iiiii" "ppppp" "iii" "ff" "pp" "s",
    "shifu_colsum_fixed": "pii" "pp" "s",
    "shifu_colsum_ws": ("ii", "l"),
    # corr_kernels.hip + gemm_kernels.hip corr_i8_kernel (K15)
    "shifu_corr_planes": "plii" "p" "ii" "pl" "pp" "s",
    "shifu_corr_gemm": "plii" "ppi" "p" "pl" "s",
    "shifu_corr_job_bytes": ("", "i"),
    # sort_kernels.hip
    "shifu_sort_ws": ("l", "l"),
    "shifu_sort_desc": "plpps",
    "shifu_gemm_set_stages": "i",
    "shifu_gemm_set_big": "i",
    "shifu_gemm_set_tune": "ii",
    "shifu_mlp_set_out_waves": "i",
    "shifu_mlp_output": "plplppl" "pplpppl" "iiiiiii" "ff" "s",
    "shifu_mlp_output_wide": "plplppl" "p" "plpl" "pppl" "iiiiiii" "ff" "s",
    "shifu_optimizer_step": "pppppp" "lii" "ffffffffff" "is",
    "shifu_optimizer_step_tf": "pppp" "li" "ffff" "ff" "p" "is",
    "shifu_cast_bf16": "plpliis",
    "shifu_split_bf16_rows": "plli" "pl" "ii" "s",
    # csv_kernels.hip
    "shifu_csv_gpu_parse": "pppl" "pi" "pl" "p" "pip" "iiP" "pp" "s",
    # autotype_kernels.hip (init -autotype on the device)
    "shifu_at_gpu_caps": "p",
    "shifu_at_gpu_codes": "pppl" "i" "pl" "p" "iiP" "iiP" "s",
    "shifu_at_gpu_apply": "pll" "pl" "pi" "pppppp" "s",
    "shifu_at_gpu_items": "pi" "ppp" "s",
    "shifu_at_gpu_hll_from_sets": "pi" "pp" "s",
    "shifu_transpose_cast": "plpiiis",
    "shifu_newline_ws_bytes": ("l", "l"),
    "shifu_newline_count_offset": ("l", "l"),
    "shifu_newline_count": "plps",
    "shifu_newline_write": "plpps",
    # svm_kernels.hip
    "shifu_svm_smo": "pl" "ppp" "pp" "ii" "dd" "pp" "s",
    # gemm_ring.hip
    "shifu_wgrad_ring": "plplpl" "iii" "pl" "s",
    "shifu_wgrad_ring_ws": ("iii", "l"),
    "shifu_ring_set_stamp": "p",
    "shifu_ring_nt_set_lab": "ip",
    "shifu_ring_nt_set_variant": "i",
    "shifu_strip_nt": "plplipl" "iii" "iiiii" "s",
    # fused head + layer-below dgrad (gemm_strip_head.hip)
    "shifu_strip_head": "plpli" "pl" "plpl" "iiii" "pi" "ppppp" "iiii" "fff" "s",
    "shifu_strip_head_rows": ("i", "i"),
    "shifu_strip_head_set_dbg_rows": "p",
    "shifu_strip_nt_set_lab": "i",
    "shifu_ring_set_mf": "i",
    "shifu_ring_set_dmamma": "i",
    # gbdt_kernels.hip
    "shifu_gbdt_hist": "pli" "ppp" "i" "pipi" "dd" "l" "i" "s",
    "shifu_gbdt_hist_root_quad": "plpppipids",
    "shifu_gbdt_hist_root_tile": "pllpppipddips",
    "shifu_gbdt_tile_bins": "pllipls",
    "shifu_gbdt_wg_stats": "pplpps",
    "shifu_gbdt_hist64": "plppp" "ipip" "ip" "iddl" "s",
    "shifu_gbdt_split": "ppipppp" "pipipp" "ppp" "iiii" "ff" "dd" "s",
    "shifu_gbdt_partition_flag": "plpl" "pppppppp" "ll" "pppp" "fi" "pppi" "s",
    "shifu_gbdt_range_index": "ppi" "pp" "s",
    "shifu_gbdt_bitrank": "pppip" "s",
    "shifu_gbdt_node_counts": "ppppipp" "pppp" "s",
    "shifu_gbdt_decide": "pii" "pp" "pp" "i" "p" "ppp" "pp" "pp" "s",
    "shifu_gbdt_items_fix": "pi" "pp" "s",
    "shifu_gbdt_leaf_window": "plpl" "ppp" "illi" "p" "pppp" "pppp" "f" "s",
    "shifu_gbdt_partition_scatter": "pppp" "ppp" "ppp" "pp" "pppp" "l" "pppi" "s",
    "shifu_gbdt_apply_tree": "plppppppp" "fi" "p" "li" "s",
    "shifu_gbdt_residual": "pppp" "p" "li" "s",
    # stats_kernels.hip
    "shifu_column_stats": "plppli" "ppii" "dd" "pipiip" "s",
    "shifu_normalize": "plli" "pppp" "pl" "s",
    "shifu_bin_codes": "plli" "pp" "pl" "s",
    "shifu_norm_codes": "plli" "pppp" "pp" "pl" "pl" "pl" "s",
    "shifu_onehot": "plli" "pp" "pl" "pl" "s",
    "shifu_lr_grad": "plli" "i" "ppp" "pp" "i" "s",
    "shifu_sensitivity": "plpl" "pp" "f" "p" "l" "iiiii" "p" "s",
    "shifu_se_perturb": "plpl" "p" "ii" "iiii" "pl" "s",
    "shifu_column_metrics": "ppp" "il" "pp" "s",
    # scoring_kernels.hip
    "shifu_tree_infer": "plll" "ppp" "pi" "pp" "iii" "pp" "s",
    "shifu_keyed_hist": "plpl" "lii" "d" "pp" "s",
    "shifu_tree_code": "plli" "ppp" "pi" "s",
    "shifu_tree_walk_coded": "pli" "pp" "p" "pi" "pp" "iiii" "pl" "p" "s",
    # wdl_kernels.hip
    "shifu_wdl_gather": "ipipipppppiipplppllls",
    "shifu_rowdot_bf16": "pllipps",
    "shifu_coldot_bf16": "ppllipps",
    "shifu_rowdot_f32_act": "pllipfiips",
    "shifu_coldot_f32": "ppllipps",
    # ga_kernels.hip
    "shifu_ga_part_floats": ("liii", "l"),
    "shifu_ga_head": "plliippppipl" "pp" "ii" "s",
    # quantile_kernels.hip
    "shifu_pack_bits": "plip" "s",
    "shifu_qprep": "pllipid" "pppp" "s",
    "shifu_qhist": "pllippid" "pipp" "pdi" "pppppp" "s",
    "shifu_qgather": "pllippid" "pipp" "d" "ppp" "ppi" "s",
}

# host runtime: name -> (argsig, restype)
RT_SIGNATURES = {
    "shifu_csv_parse": ("plPipPi", "p"),
    "shifu_csv_scan": ("plPipPi", "p"),
    "shifu_csv_fill": ("ppl", "i"),
    "shifu_csv_nrows": ("p", "l"),
    "shifu_csv_bad_rows": ("p", "l"),
    "shifu_csv_numeric": ("pip", "i"),
    "shifu_csv_codes": ("pip", "i"),
    "shifu_csv_dict": ("pipl", "l"),
    "shifu_csv_dict_size": ("pi", "l"),
    "shifu_csv_free": ("p", None),
    "shifu_spdt_bins": ("pplipl", "l"),
    "shifu_munropat_bins": ("plipl", "l"),
    "shifu_format_rows": ("lipppppplp", "l"),
    "shifu_format_rows_sep": ("lipppppplpPi", "l"),
    "shifu_join_lines": ("plPiipplpli", "l"),
    "shifu_merge_runs": ("ippppP", "l"),
    "shifu_gather_lines": ("ppplPp", "l"),
    "shifu_eval_set_flush_bytes": ("l", "l"),
    "shifu_gen_csv": ("Pliildii", "i"),
    "shifu_gen_strong_cols": ("iip", "i"),
    "shifu_parse_fields": ("ppLp", "l"),
    "shifu_gather_fields": ("pplipPpl", "l"),
    # autotype_scan.cpp (init -autotype)
    "shifu_at_new": ("iiPPP", "p"),
    "shifu_at_feed": ("pplpi", "l"),
    "shifu_at_counts": ("pp", "l"),
    "shifu_at_exact": ("pipl", "l"),
    "shifu_at_hll_p": ("", "i"),
    "shifu_at_exact_cap": ("", "i"),
    "shifu_at_hll": ("pp", "i"),
    "shifu_at_hll_estimate": ("p", "d"),
    "shifu_at_items": ("pipl", "l"),
    "shifu_at_skipped": ("p", "l"),
    "shifu_at_free": ("p", None),
}


class NativeUnavailable(RuntimeError):
    pass


def _bind(lib, sigs):
    for name, sig in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise NativeUnavailable(f"symbol {name} missing from {lib._name}; rebuild with "
                                    f"`python -m shifu_amd.build_native`")
        res = "i"
        if isinstance(sig, tuple):
            sig, res = sig
        fn.argtypes = [_T[c] for c in sig]
        fn.restype = None if res is None else _T[res]


def register_hip(sigs: dict):
    HIP_SIGNATURES.update(sigs)


def register_rt(sigs: dict):
    RT_SIGNATURES.update(sigs)


def hip():
    """The HIP kernel library (raises loudly when missing)."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            if not HIP_LIB.exists():
                raise NativeUnavailable(
                    f"{HIP_LIB} not built: run `python -m shifu_amd.build_native` (hipcc gfx950)")
            lib = ctypes.CDLL(str(HIP_LIB), mode=ctypes.RTLD_GLOBAL)
            _bind(lib, HIP_SIGNATURES)
            # SHIFU_GEMM_TUNE="key=value,...": GEMM dispatch knobs (gemm_kernels.hip
            # shifu_gemm_set_tune; e.g. 12=0 turns the persistent ring forward off) for A/B runs
            for kv in filter(None, os.environ.get("SHIFU_GEMM_TUNE", "").split(",")):
                k, v = kv.split("=")
                if lib.shifu_gemm_set_tune(int(k), int(v)) != 0:
                    raise ValueError(f"SHIFU_GEMM_TUNE: bad knob {kv}")
            _hip = lib
    return _hip


def rt(build_if_missing: bool = True):
    """The host C++ runtime library (built on demand with g++, seconds), or None."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            if not RT_LIB.exists() and build_if_missing and os.environ.get("SHIFU_NO_RT_BUILD") != "1":
                try:
                    from ..build_native import build_rt
                    build_rt()
                except Exception:   # pragma: no cover - toolchain missing
                    return None
            if RT_LIB.exists():
                lib = ctypes.CDLL(str(RT_LIB))
                _bind(lib, RT_SIGNATURES)
                _rt = lib
    return _rt


def hip_available() -> bool:
    try:
        hip()
        return True
    except (NativeUnavailable, OSError):
        return False


def check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"native call {name} failed with code {rc}")


def call_hip(name: str, *args):
    """Launch ``name``.  torch tensors may be passed directly: they are converted to device
    pointers here and stay referenced until the launch has been enqueued (never pass
    ``tmp().data_ptr()`` - the temporary is freed and its block re-issued by the caching
    allocator before the kernel runs)."""
    fn = getattr(hip(), name)
    keep = args
    conv = [a.data_ptr() if hasattr(a, "data_ptr") else a for a in args]
    rc = fn(*conv)
    del keep
    if rc != 0:
        raise RuntimeError(f"HIP kernel launcher {name} returned {rc} (bad shape or HIP error)")
    return rc


def stream_of(t=None):
    """Current torch HIP stream handle as an int (hipStream_t)."""
    import torch
    dev = t.device if t is not None else None
    return torch.cuda.current_stream(dev).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def require_gpu_native():
    """On a GPU run the HIP library must be present; raise otherwise."""
    if os.environ.get("SHIFU_ALLOW_TORCH_FALLBACK") == "1":
        return hip_available()
    hip()
    return True
