"""Per-step config validation (C3): ``ModelInspector.probe`` (J/core/validator/ModelInspector.java:93-200):
the meta-driven item checks of ``MetaFactory`` first (``config/meta.py``), then the step checks,
``checkTrainSetting`` (:451-938) included, plus ``BasicModelProcessor.checkAlgorithmParam``
defaults (J/core/processor/BasicModelProcessor.java:404-494)."""
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
    from .meta import validate_config
    for cause in validate_config(mc):         # checkMeta: a meta violation ends the probe
        r.fail(cause)
    if not r:
        return r
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
    if t.get("epochsPerIteration") is not None and int(t.get("epochsPerIteration")) <= 0:
        r.fail("'epochsPerIteration' should be larger than 0 if set.")
    if t.get("convergenceThreshold") is not None and float(t.get("convergenceThreshold")) < 0:
        r.fail("'convergenceThreshold' should be larger than or equal to 0 if set.")
    wtc = t.get("workerThreadCount")
    if wtc is not None and (int(wtc) <= 0 or int(wtc) > 32):
        r.fail("'workerThreadCount' should be in (0, 32] if set.")
    if mc.is_multiclass():
        method = str(t.get("multiClassifyMethod", "NATIVE")).upper()
        if method in ("ONEVSALL", "ONEVSREST") and alg not in ("GBT", "RF", "NN"):
            r.fail("OneVSAll multiple classification is only effective in gradient boosted trees (GBT) or "
                   "random forest (RF) or Neural Network (NN) training method.")
        if method == "NATIVE" and alg not in ("NN", "RF"):
            r.fail("Native multiple classification is only effective in neural network (nn) or random forest "
                   "(rf) training method.")
    p = mc.params or {}
    from .meta import has_grid
    if not has_grid(mc):
        _check_params(alg, p, r)
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


def _f(v):
    try:
        return None if v is None else float(v)
    except (TypeError, ValueError):
        return None


def _check_params(alg: str, p: dict, r: ValidateResult) -> None:
    """Value ranges of ``checkTrainSetting`` (ModelInspector.java:527-938) for concrete params."""
    lr = _f(p.get("LearningRate"))
    if lr is not None and lr <= 0:
        r.fail("Learning rate should be larger than 0.")
    if alg == "NN":
        ld = _f(p.get("LearningDecay"))
        if ld is not None and (ld < 0 or ld >= 1):
            r.fail("Learning decay should be in [0, 1) if set.")
        mb = _f(p.get("MiniBatchs"))
        if mb is not None and (mb <= 0 or mb > 1000):
            r.fail("MiniBatchs should be in (0, 1000] if set.")
        mom = _f(p.get("Momentum"))
        if mom is not None and mom <= 0:
            r.fail("Momentum should be larger than 0 if set.")
        for k in ("AdamBeta1", "AdamBeta2"):
            b = _f(p.get(k))
            if b is not None and (b <= 0 or b >= 1):
                r.fail(f"{k} should be in (0, 1) if set.")
    if alg in ("NN", "GBT", "RF"):
        dr = _f(p.get("DropoutRate"))
        if dr is not None and (dr < 0 or dr >= 1):
            r.fail("Dropout rate should be in [0, 1) if set.")
    if alg in ("GBT", "RF"):
        fss = p.get("FeatureSubsetStrategy")
        if fss is None:
            r.fail("'FeatureSubsetStrategy' should not be null for GBT/RF.")
        else:
            v = _f(fss)
            if v is not None:
                if v <= 0 or v > 1:
                    r.fail("'FeatureSubsetStrategy' as a number should be in (0, 1].")
            elif str(fss).upper() not in ("ALL", "HALF", "ONETHIRD", "TWOTHIRDS", "SQRT", "LOG2", "AUTO"):
                r.fail(f"'FeatureSubsetStrategy' {fss} is not one of ALL, HALF, ONETHIRD, TWOTHIRDS, SQRT, "
                       "LOG2, AUTO or a number in (0, 1].")
        md, ml = p.get("MaxDepth"), p.get("MaxLeaves")
        if md is None and ml is None:
            r.fail("'MaxDepth' or 'MaxLeaves' should be set for GBT/RF.")
        if ml is not None and int(ml) <= 0:
            r.fail("'MaxLeaves' should be larger than 0 if set.")
        vt = _f(p.get("ValidationTolerance"))
        if vt is not None and (vt < 0 or vt >= 1):
            r.fail("'ValidationTolerance' should be in [0, 1) if set.")
        msm = p.get("MaxStatsMemoryMB")
        if msm is not None and int(msm) <= 0:
            r.fail("'MaxStatsMemoryMB' should be larger than 0 if set.")
        mipn = p.get("MinInstancesPerNode")
        if mipn is not None and int(mipn) <= 0:
            r.fail("'MinInstancesPerNode' should be larger than 0 if set.")
        tn = p.get("TreeNum")
        if tn is not None and (int(tn) <= 0 or int(tn) > 10000):
            r.fail("'TreeNum' should be in (0, 10000] if set.")
        mig = _f(p.get("MinInfoGain"))
        if mig is not None and mig < 0:
            r.fail("'MinInfoGain' should be larger than or equal to 0 if set.")
