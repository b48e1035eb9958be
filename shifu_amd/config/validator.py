"""Per-step config validation (C3) - subset of ``ModelInspector.probe``
(J/core/validator/ModelInspector.java:93, checkTrainSetting :451-938) plus
``BasicModelProcessor.checkAlgorithmParam`` defaults (J/core/processor/BasicModelProcessor.java:404-494)."""
from __future__ import annotations

import os

from .enums import ALGORITHMS, NORM_TYPES


class ValidateResult:
    def __init__(self):
        self.status = True
        self.causes: list[str] = []

    def fail(self, msg):
        self.status = False
        self.causes.append(msg)

    def __bool__(self):
        return self.status

    def __repr__(self):
        return f"ValidateResult({self.status}, {self.causes})"


STEPS = ("INIT", "STATS", "VARSELECT", "NORMALIZE", "TRAIN", "POSTTRAIN", "EVAL", "EXPORT", "COMBO", "ENCODE")


def probe(mc, step: str) -> ValidateResult:
    r = ValidateResult()
    step = step.upper()
    basic = mc.basic
    if not basic.get("name"):
        r.fail("basic.name must not be empty")
    ds = mc.dataSet
    if step in ("INIT", "STATS", "NORMALIZE", "VARSELECT", "TRAIN"):
        if not ds.get("dataPath"):
            r.fail("dataSet.dataPath must not be empty")
        elif not os.path.exists(mc.resolve(ds.get("dataPath"))):
            r.fail(f"dataSet.dataPath {ds.get('dataPath')} does not exist")
        if not ds.get("targetColumnName"):
            r.fail("dataSet.targetColumnName must not be empty")
        pos, neg = set(mc.pos_tags), set(mc.neg_tags)
        if pos & neg:
            r.fail("posTags and negTags overlap: " + ",".join(sorted(pos & neg)))
    if step == "STATS":
        mnb = mc.stats.get("maxNumBin", 10)
        if int(mnb) <= 0:
            r.fail("stats.maxNumBin must be > 0")
        sr = float(mc.stats.get("sampleRate", 1.0))
        if not 0 < sr <= 1:
            r.fail("stats.sampleRate must be in (0, 1]")
    if step == "NORMALIZE":
        nt = mc.normalize.get("normType", "ZSCALE")
        if str(nt).upper() not in NORM_TYPES:
            r.fail(f"normalize.normType {nt} is not one of {NORM_TYPES}")
        if float(mc.normalize.get("stdDevCutOff", 6.0)) <= 0:
            r.fail("normalize.stdDevCutOff must be > 0")
    if step == "VARSELECT":
        fb = str(mc.varSelect.get("filterBy", "KS")).upper()
        if fb not in ("KS", "IV", "MIX", "PARETO", "SE", "ST", "SR", "FI", "V", "VOTED", "R", "C"):
            r.fail(f"varSelect.filterBy {fb} is not supported")
    if step == "TRAIN":
        check_train(mc, r)
    if step == "EVAL":
        for e in mc.evals:
            if not e.get("name"):
                r.fail("eval name must not be empty")
            eds = e.get("dataSet")
            if eds is None or not eds.get("dataPath"):
                r.fail(f"eval {e.get('name')}: dataSet.dataPath must not be empty")
    return r


def check_train(mc, r: ValidateResult):
    t = mc.train
    alg = str(t.get("algorithm", "NN")).upper()
    if alg not in ALGORITHMS:
        r.fail(f"train.algorithm {alg} is not supported")
    if int(t.get("baggingNum", 1)) <= 0:
        r.fail("train.baggingNum must be > 0")
    vr = float(t.get("validSetRate", 0.2))
    if not 0 <= vr < 1:
        r.fail("train.validSetRate must be in [0, 1)")
    bsr = float(t.get("baggingSampleRate", 1.0))
    if not 0 < bsr <= 1:
        r.fail("train.baggingSampleRate must be in (0, 1]")
    if int(t.get("numTrainEpochs", 100)) <= 0:
        r.fail("train.numTrainEpochs must be > 0")
    p = mc.params or {}
    if alg == "NN":
        nl = p.get("NumHiddenLayers", 1)
        nodes = p.get("NumHiddenNodes", [])
        acts = p.get("ActivationFunc", [])
        if not isinstance(nl, list):
            try:
                nl_i = int(nl)
            except (TypeError, ValueError):
                nl_i = -1
            if nl_i < 0:
                r.fail("NumHiddenLayers must be >= 0")
            elif isinstance(nodes, list) and len(nodes) != nl_i:
                r.fail("NumHiddenNodes size must equal NumHiddenLayers")
            elif isinstance(acts, list) and len(acts) != nl_i:
                r.fail("ActivationFunc size must equal NumHiddenLayers")
        prop = str(p.get("Propagation", "R")).upper()
        if prop not in ("B", "Q", "M", "R", "ADAM", "ADAGRAD", "RMSPROP", "MOMENTUM", "NESTEROV", "S"):
            r.fail(f"Propagation {prop} is not supported")
        if prop == "S":
            r.fail("Propagation S (SCG) is not supported in distributed NN training")
    if alg in ("GBT", "RF"):
        md = int(p.get("MaxDepth", 7))
        if md <= 0 or md > 20:
            r.fail("MaxDepth must be in [1, 20]")
        imp = str(p.get("Impurity", "variance")).lower()
        if imp not in ("variance", "friedmanmse", "entropy", "gini"):
            r.fail(f"Impurity {imp} is not supported")
        if alg == "GBT" and imp in ("entropy", "gini"):
            r.fail("GBT only supports variance / friedmanmse impurity")
        loss = str(p.get("Loss", "squared")).lower()
        if loss not in ("squared", "halfgradsquared", "absolute", "log"):
            r.fail(f"Loss {loss} is not supported")
    if alg == "LR" and mc.is_multiclass() and not mc.is_one_vs_all():
        r.fail("LR supports multi-class only with multiClassifyMethod ONEVSALL")
    kf = int(t.get("numKFold", -1))
    if kf > 20:
        r.fail("numKFold must be <= 20")
    return r
