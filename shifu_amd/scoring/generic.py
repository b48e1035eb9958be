"""Generic models (I5): externally trained models scored inside a Shifu model set.

The reference reads ``models/*.json`` ``GenericModelConfig`` files (``{"inputnames": [...],
"properties": {"algorithm": ..., ...}}``, J/container/obj/GenericModelConfig.java:34-83) when
``ModelConfig.train.algorithm`` is ``generic`` / ``tensorflow`` and wraps a ``Computable``
(``init(config)`` / ``compute(MLData)`` / ``releaseResource()``, J/core/Computable.java,
J/core/GenericModel.java:30-90; loader J/util/ModelSpecLoaderUtils.java:182-250).

Here the same JSON selects an implementation by ``properties.algorithm``:

* ``python``            - ``properties.class = "module:Class"`` (module importable, or a ``.py``
                          file next to the JSON): an object with ``init(config: dict)``,
                          ``compute(X: np.ndarray[N, n_inputs]) -> [N] or [N, k]`` and optional
                          ``release()``.  The in-process analogue of the Java ``Computable``.
* ``safetensors_mlp``   - a dense MLP stored as safetensors (``W0, b0, W1, b1, ...``; ``W_l`` is
                          [out, in]) plus ``properties.activations``; scored on the GPU with
                          torch GEMMs.  Loaded with the safetensors reader (no code execution).
* ``tensorflow``        - TensorFlow SavedModels need a TensorFlow runtime, which this
                          MI355X build does not ship; loading raises with that message.

Inputs are the ColumnConfig-normalized values of ``inputnames`` (default: the model set's
selected columns, in ColumnConfig order), as the reference feeds its TF models.
"""
from __future__ import annotations

import importlib
import importlib.util
import json
import os

import numpy as np
import torch

GENERIC_ALGORITHMS = ("generic", "tensorflow")


class GenericModel:
    """Loaded generic model: ``compute(X) -> [N, n_out]`` float64."""

    def __init__(self, path: str, config: dict, impl, n_out: int = 1):
        self.path, self.config, self.impl, self.n_out = path, config, impl, n_out

    @property
    def input_names(self):
        return list(self.config.get("inputnames") or [])

    def compute(self, X: np.ndarray) -> np.ndarray:
        out = np.asarray(self.impl.compute(np.asarray(X, dtype=np.float32)), dtype=np.float64)
        return out[:, None] if out.ndim == 1 else out

    def release(self):
        rel = getattr(self.impl, "release", None) or getattr(self.impl, "releaseResource", None)
        if rel:
            rel()


class SafetensorsMLP:
    """Dense MLP from a safetensors file (the TF/Keras-export-free generic model)."""

    def init(self, config: dict):
        from safetensors.torch import load_file
        from ..models.nn import act_fwd, norm_act
        props = config.get("properties", {})
        base = props.get("modelpath") or os.path.dirname(config["_path"])
        f = props.get("weights", "model.safetensors")
        t = load_file(f if os.path.isabs(f) else os.path.join(base, f))
        self.dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        n = 0
        while f"W{n}" in t:
            n += 1
        if n == 0:
            raise ValueError("safetensors_mlp: no W0 tensor")
        self.W = [t[f"W{i}"].float().to(self.dev) for i in range(n)]
        self.b = [t[f"b{i}"].float().to(self.dev) if f"b{i}" in t else None for i in range(n)]
        acts = props.get("activations") or ["sigmoid"] * n
        self.acts = [norm_act(a) for a in acts] + ["sigmoid"] * max(0, n - len(acts))
        self._act = act_fwd

    @torch.no_grad()
    def compute(self, X: np.ndarray) -> np.ndarray:
        a = torch.as_tensor(X, dtype=torch.float32, device=self.dev)
        for W, b, act in zip(self.W, self.b, self.acts):
            z = a @ W.t()
            if b is not None:
                z = z + b
            a = self._act(act, z)
        return a.double().cpu().numpy()


def _python_impl(spec: str, base_dir: str):
    mod_name, _, cls_name = spec.partition(":")
    if not cls_name:
        raise ValueError(f"generic python model: class must be 'module:Class', got {spec!r}")
    local = os.path.join(base_dir, mod_name + ".py")
    if os.path.exists(local):
        sp = importlib.util.spec_from_file_location(f"shifu_generic_{mod_name}", local)
        mod = importlib.util.module_from_spec(sp)
        sp.loader.exec_module(mod)
    else:
        mod = importlib.import_module(mod_name)
    return getattr(mod, cls_name)()


def load_generic(path: str) -> GenericModel:
    with open(path) as fh:
        cfg = json.load(fh)
    cfg["_path"] = path
    props = cfg.setdefault("properties", {})
    props.setdefault("modelpath", os.path.dirname(os.path.abspath(path)))
    alg = str(props.get("algorithm", "")).lower()
    if alg == "python":
        impl = _python_impl(props.get("class", ""), props["modelpath"])
    elif alg in ("safetensors_mlp", "mlp"):
        impl = SafetensorsMLP()
    elif alg == "tensorflow":
        raise RuntimeError("generic model algorithm 'tensorflow' needs a TensorFlow runtime, which is not "
                           "part of this build; export the network as safetensors_mlp or wrap it as a "
                           "'python' generic model")
    else:
        raise RuntimeError(f"Algorithm: {alg} is not supported in generic model yet.")
    impl.init(cfg)
    return GenericModel(path, cfg, impl, int(props.get("n_out", 1)))


def find_generic_models(models_dir: str):
    """``models/*.json`` generic model configs and ``models/<name>/GenericModelConfig.json``
    model directories (the layout the reference's TF trainer writes; checkpoint directories
    ``<name>-checkpoint-<epoch>`` are skipped), sorted by path."""
    import glob
    cands = glob.glob(os.path.join(models_dir, "*.json"))
    cands += [p for p in glob.glob(os.path.join(models_dir, "*", "GenericModelConfig.json"))
              if "-checkpoint-" not in os.path.basename(os.path.dirname(p))]
    return sorted(p for p in cands if _is_generic_config(p))


def _is_generic_config(path: str) -> bool:
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return False
    return isinstance(d, dict) and isinstance(d.get("properties"), dict) and "algorithm" in d["properties"]
