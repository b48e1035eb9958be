"""Synthetic tabular data sets (no network, no downloaded data): ``|``-delimited part files with
a ``.pig_header``, numeric + categorical columns, a weight column and a binary (or multi-class)
tag — the same shape of input the reference's example model sets use."""
from __future__ import annotations

import os

import numpy as np


def make_dataset(root: str, n_rows: int = 2000, n_num: int = 20, n_cat: int = 3, seed: int = 0,
                 n_classes: int = 2, missing_rate: float = 0.02, n_eval: int | None = None):
    """Write ``root/DataSet1`` and ``root/EvalSet1``; returns dict of paths and tag lists."""
    rng = np.random.default_rng(seed)
    coef = rng.normal(size=n_num)
    cat_eff = [rng.normal(size=5) for _ in range(n_cat)]

    def rows(n, rs):
        X = rs.normal(size=(n, n_num))
        C = rs.integers(0, 5, size=(n, n_cat))
        z = X @ coef * 0.6 + sum(cat_eff[j][C[:, j]] for j in range(n_cat)) + rs.normal(size=n) * 0.8
        if n_classes == 2:
            tag = np.where(z > 0, "M", "B")
        else:
            qs = np.quantile(z, np.linspace(0, 1, n_classes + 1)[1:-1])
            tag = np.array([f"c{k}" for k in np.searchsorted(qs, z)])
        w = rs.uniform(0.5, 2.0, size=n)
        lines = []
        for i in range(n):
            vals = [f"id{i}", tag[i], f"{w[i]:.4f}"]
            for j in range(n_num):
                vals.append("" if rs.random() < missing_rate else f"{X[i, j]:.5f}")
            for j in range(n_cat):
                vals.append("" if rs.random() < missing_rate else f"k{C[i, j]}")
            lines.append("|".join(vals))
        return lines
    header = ["id", "diagnosis", "wgt"] + [f"num_{j}" for j in range(n_num)] + [f"cat_{j}" for j in range(n_cat)]
    out = {}
    for name, n, s in (("DataSet1", n_rows, seed + 1), ("EvalSet1", n_eval or max(200, n_rows // 4), seed + 2)):
        d = os.path.join(root, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "part-00000"), "w") as f:
            f.write("\n".join(rows(n, np.random.default_rng(s))) + "\n")
        with open(os.path.join(d, ".pig_header"), "w") as f:
            f.write("|".join(header) + "\n")
        out[name] = d
    out["header"] = header
    out["meta"] = ["id"]
    out["categorical"] = [f"cat_{j}" for j in range(n_cat)]
    out["pos"], out["neg"] = (["M"], ["B"]) if n_classes == 2 else ([f"c{k}" for k in range(n_classes)], [])
    return out


def make_model_set(parent: str, name: str = "demo", alg: str = "NN", n_rows: int = 2000, seed: int = 0,
                   n_classes: int = 2, **kw):
    """``shifu new`` + point the data set / eval set at freshly generated synthetic data."""
    from ..config.model_config import ModelConfig
    from ..steps.create import create_model_set
    root = create_model_set(name, alg, parent=parent)
    ds = make_dataset(os.path.join(root, "data"), n_rows=n_rows, seed=seed, n_classes=n_classes, **kw)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    for sec, key in ((mc.dataSet, "DataSet1"), (mc.evals[0].dataSet, "EvalSet1")):
        sec["dataPath"] = ds[key]
        sec["headerPath"] = os.path.join(ds[key], ".pig_header")
        sec["targetColumnName"] = "diagnosis"
        sec["posTags"] = ds["pos"]
        sec["negTags"] = ds["neg"]
        sec["weightColumnName"] = "wgt"
    with open(os.path.join(root, "columns", "meta.column.names"), "w") as f:
        f.write("\n".join(ds["meta"]) + "\n")
    with open(os.path.join(root, "columns", "categorical.column.names"), "w") as f:
        f.write("\n".join(ds["categorical"]) + "\n")
    if n_classes > 2:
        mc.train["multiClassifyMethod"] = "NATIVE"
    mc.save()
    return root
