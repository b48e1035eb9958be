"""Meta-driven ModelConfig validation (C3): the item-level rules of ``MetaFactory.validate``
(J/container/meta/MetaFactory.java:125-510) over a schema table of every ModelConfig item.

The reference loads ``R/store/ModelConfigMeta.json`` into a flat warehouse keyed
``group#name[#sub...]`` and checks every bean field against it.  Here the schema is a declarative
table (``SCHEMA`` below, written against this package's enums), flattened the same way, and
``validate_config`` walks the ModelConfig dicts with the same per-type rules:

* ``text``: optional min/max length; options matched case-insensitively;
* ``integer`` / ``number``: must parse; options must match (numbers with 1e-6 tolerance);
* ``boolean``: must be present and true/false;
* ``list``: every element checked against the element meta (``key#dummy``) or, for object
  lists, field by field;  ``map``: every entry checked against ``key#<entry key>``: an entry
  without meta info is an error (a typo in ``train.params`` is reported, as in the reference);
* bean fields without meta (unknown JSON properties) are ignored, as Jackson drops them;
* with a grid search (``train.params`` holding lists of candidates or ``gridConfigFile``)
  ``train#params#*`` items are not checked (``MetaFactory.filterOut``).
"""
from __future__ import annotations

from .enums import ALGORITHMS, NORM_TYPES

OK = "OK"

_ACTS = ["Sigmoid", "Tanh", "PTanh", "Log", "Sin", "Linear", "ReLU", "LeakyReLU", "Swish"]

# (name, type, extra) with extra: options / min / max / element (list element meta or map/object fields)
SCHEMA = {
    "basic": [
        ("name", "text", {"min": 1}), ("author", "text", {"min": 0}), ("description", "text", {}),
        ("runMode", "text", {"options": ["local", "mapred", "dist"]}), ("version", "text", {}),
        ("postTrainOn", "boolean", {}),
        ("customPaths", "map", {"fields": [("hdfsModelSetPath", "text", {})]}),
    ],
    "dataSet": [
        ("source", "text", {"options": ["HDFS", "LOCAL", "S3"]}), ("dataPath", "text", {}),
        ("validationDataPath", "text", {}), ("dataDelimiter", "text", {"min": 1, "max": 20}),
        ("headerPath", "text", {}), ("headerDelimiter", "text", {}), ("filterExpressions", "text", {}),
        ("validationFilterExpressions", "text", {}), ("weightColumnName", "text", {}),
        ("targetColumnName", "text", {}),
        ("posTags", "list", {"element": ("text", {})}), ("negTags", "list", {"element": ("text", {})}),
        ("missingOrInvalidValues", "list", {"element": ("text", {})}),
        ("metaColumnNameFile", "text", {}), ("autoType", "boolean", {}), ("autoTypeThreshold", "number", {}),
        ("hybridColumnNameFile", "text", {}), ("segExpressionFile", "text", {}),
        ("categoricalColumnNameFile", "text", {}),
    ],
    "stats": [
        ("maxNumBin", "integer", {}), ("cateMaxNumBin", "integer", {}),
        ("binningMethod", "text", {"options": ["EqualNegative", "EqualPositive", "EqualTotal", "EqualInterval",
                                               "WeightEqualNegative", "WeightEqualPositive", "WeightEqualTotal",
                                               "WeightEqualInterval"]}),
        ("sampleRate", "number", {}), ("sampleNegOnly", "boolean", {}), ("numericalValueThreshold", "number", {}),
        ("binningAutoTypeEnable", "boolean", {}), ("binningAutoTypeThreshold", "integer", {}),
        ("binningMergeEnable", "boolean", {}),
        ("binningAlgorithm", "text", {"options": ["Native", "SPDTI", "SPDT", "MunroPat", "MunroPatI",
                                                  "DynamicBinning"]}),
        ("psiColumnName", "text", {}),
    ],
    "varSelect": [
        ("forceEnable", "boolean", {}), ("forceSelectColumnNameFile", "text", {}),
        ("candidateColumnNameFile", "text", {}), ("forceRemoveColumnNameFile", "text", {}),
        ("filterEnable", "boolean", {}), ("filterNum", "integer", {}), ("filterOutRatio", "number", {}),
        ("epsilons", "numberarray", {}),
        ("filterBy", "text", {"options": ["ks", "iv", "mix", "pareto", "SE", "ST", "V", "FI"]}),
        ("votedVariablesSelection", "boolean", {}), ("autoFilterEnable", "boolean", {}),
        ("missingRateThreshold", "number", {}), ("correlationThreshold", "number", {}),
        ("minIvThreshold", "number", {}), ("minKsThreshold", "number", {}),
        ("postCorrelationMetric", "text", {"options": ["KS", "IV", "SE"]}),
        ("params", "map", {"fields": [("worker_sample_rate", "number", {}), ("population_multiply_cnt", "integer", {}),
                                      ("population_live_size", "integer", {}), ("expect_variable_cnt", "integer", {}),
                                      ("hybrid_percent", "number", {}), ("mutation_percent", "number", {})]}),
    ],
    "normalize": [
        ("normType", "text", {"options": list(NORM_TYPES)}), ("stdDevCutOff", "number", {}),
        ("sampleRate", "number", {}), ("isParquet", "boolean", {}), ("sampleNegOnly", "boolean", {}),
    ],
    "train": [
        ("baggingNum", "integer", {}), ("baggingWithReplacement", "boolean", {}), ("baggingSampleRate", "number", {}),
        ("baggingSampleSeed", "integer", {}), ("validSetRate", "number", {}), ("sampleNegOnly", "boolean", {}),
        ("trainOnDisk", "boolean", {}), ("numKFold", "integer", {}), ("fixInitInput", "boolean", {}),
        ("stratifiedSample", "boolean", {}), ("numTrainEpochs", "integer", {}),
        ("convergenceThreshold", "number", {}), ("zkServers", "text", {}), ("epochsPerIteration", "integer", {}),
        ("isContinuous", "boolean", {}), ("isCrossOver", "boolean", {}), ("workerThreadCount", "integer", {}),
        ("multiClassifyMethod", "text", {"options": ["NATIVE", "ONEVSALL", "ONEVSREST", "ONEVSONE"]}),
        ("upSampleWeight", "number", {}),
        ("algorithm", "text", {"options": [a if a not in ("TENSORFLOW", "GENERIC") else
                                           {"TENSORFLOW": "Tensorflow", "GENERIC": "generic"}[a]
                                           for a in ALGORITHMS] + ["SVM", "DT"]}),
        ("gridConfigFile", "text", {}),
        ("params", "map", {"fields": [
            ("NumHiddenLayers", "integer", {}), ("TF.alg", "text", {}),
            ("ActivationFunc", "list", {"element": ("text", {"options": _ACTS})}),
            ("CheckpointInterval", "integer", {}),
            ("NumHiddenNodes", "list", {"element": ("integer", {})}),
            ("NumEmbedColumnIds", "list", {"element": ("integer", {})}),
            ("LearningRate", "number", {}), ("WDLL2Reg", "float", {}),
            ("TF.optimizer", "text", {"options": ["adam", "gradientDescent", "RMSProp"]}),
            ("TF.loss", "text", {"options": ["squared", "absolute", "log"]}),
            ("Momentum", "number", {}), ("AdamBeta1", "number", {}), ("AdamBeta2", "number", {}),
            ("RegularizedConstant", "number", {}),
            ("WeightInitializer", "text", {"options": ["default", "gaussian", "Xavier", "He", "Lecun"]}),
            ("L1orL2", "text", {}), ("MaxDepth", "integer", {}), ("MaxLeaves", "integer", {}),
            ("MaxBatchSplitSize", "integer", {}), ("MinInstancesPerNode", "integer", {}),
            ("MinInfoGain", "number", {}), ("MaxStatsMemoryMB", "integer", {}), ("TreeNum", "integer", {}),
            ("Impurity", "text", {"options": ["variance", "friedmanmse", "entropy", "gini"]}),
            ("FeatureSubsetStrategy", "text", {}), ("EnableEarlyStop", "boolean", {}),
            ("Loss", "text", {"options": ["squared", "halfgradsquared", "absolute", "log"]}),
            ("LearningDecay", "number", {}), ("DropoutRate", "number", {}), ("MiniBatchs", "number", {}),
            ("ValidationTolerance", "number", {}),
            ("Propagation", "text", {"options": ["Q", "B", "M", "R", "S", "Adam", "AdaGrad", "RMSProp", "Nesterov",
                                                 "Momentum"]}),
            ("IsELM", "boolean", {}), ("GBTSampleWithReplacement", "boolean", {}), ("Kernel", "text", {}),
            ("Const", "number", {}), ("Gamma", "number", {}),
            ("FixedLayers", "list", {"element": ("integer", {})}), ("FixedBias", "boolean", {}),
            ("OutputActivationFunc", "text", {"options": ["Linear", "ReLU", "LeakyReLU", "Swish"]}),
            # parameters the reference's trainers read (CommonConstants / WDLMaster, WDLWorker,
            # DTMaster) that its meta store lacks: accepted so a working reference config validates
            ("NumEmbedOuputs", "integer", {}), ("SUBSETFEATURES", "text", {}), ("Optimizer", "text", {}),
        ]}),
        ("customPaths", "map", {"fields": [(k, "text", {}) for k in (
            "preTrainStatsPath", "normalizedDataPath", "normalizedValidationDataPath", "cleanedDataPath",
            "cleanedValidationDataPath", "selectedRawDataPath", "trainScoresPath", "binAvgScorePath")]}),
    ],
    "evals": [
        ("name", "text", {"min": 1}),
        ("dataSet", "object", {"fields": [
            ("source", "text", {"options": ["HDFS", "LOCAL", "S3"]}), ("dataPath", "text", {}),
            ("testDataPath", "text", {}), ("dataDelimiter", "text", {"min": 1, "max": 20}),
            ("headerPath", "text", {}), ("headerDelimiter", "text", {}), ("filterExpressions", "text", {}),
            ("weightColumnName", "text", {}), ("targetColumnName", "text", {}),
            ("posTags", "list", {"element": ("text", {})}), ("negTags", "list", {"element": ("text", {})})]}),
        ("performanceBucketNum", "integer", {}), ("scoreScale", "number", {}), ("gbtConvertToProb", "boolean", {}),
        ("normAllColumns", "boolean", {}),
        ("gbtScoreConvertStrategy", "text", {"options": ["RAW", "OLD_SIGMOID", "SIGMOID", "CUTOFF", "HALF_CUTOFF",
                                                         "MAXMIN"]}),
        ("performanceScoreSelector", "text", {}), ("scoreMetaColumnNameFile", "text", {}),
        ("customPaths", "map", {"fields": [(k, "text", {}) for k in (
            "modelsPath", "scorePath", "confusionMatrixPath", "performancePath")]}),
    ],
}


def _flatten() -> dict:
    wh = {}

    def add(key, typ, extra):
        wh[key] = (typ, extra)
        if typ == "list" and "element" in extra:
            et, ex = extra["element"]
            add(key + "#dummy", et, ex)
        for sub in extra.get("fields", []):
            add(key + "#" + sub[0], sub[1], sub[2])
    for g, items in SCHEMA.items():
        for name, typ, extra in items:
            add(g + "#" + name, typ, extra)
    return wh


WAREHOUSE = _flatten()


def _num(v, cast):
    try:
        return cast(str(v).strip()) if not isinstance(v, bool) else None
    except (TypeError, ValueError):
        return None


def check_item(key: str, value, grid: bool = False) -> str:
    """``MetaFactory.validate(isGridSearch, itemKey, itemValue)``: OK or the error message."""
    if grid and key.startswith("train#params#"):
        return OK
    meta = WAREHOUSE.get(key)
    if meta is None:
        return key + " - not found meta info."
    typ, ex = meta
    opts = ex.get("options")
    if typ == "text":
        s = None if value is None else str(value)
        if ex.get("max") is not None and s is not None and len(s) > ex["max"]:
            return f"{key} - the length of value exceeds the max length : {ex['max']}"
        if ex.get("min") is not None and (s is None or len(s) < ex["min"]):
            return f"{key} - then shouldn't be null" if s is None else \
                f"{key} - the length of value less than min length : {ex['min']}"
        if opts and (s is None or s.lower() not in [o.lower() for o in opts]):
            return f"{key} - the value couldn't be found in the option value list - {', '.join(opts)}"
    elif typ in ("integer", "int", "number", "float"):
        if value is None:
            return f"{key} - the value couldn't be null." if opts else OK
        cast = int if typ in ("integer", "int") else float
        v = _num(value, cast)
        if v is None:
            return f"{key} - the value is not {'integer' if cast is int else 'number'} format."
        if opts and not any(abs(v - cast(o)) <= 1e-6 for o in opts):
            return f"{key} - the value couldn't be found in the option value list - {opts}"
    elif typ == "boolean":
        if value is None:
            return f"{key} - the value couldn't be null. Only true/false are perimited."
        if str(value).lower() not in ("true", "false"):
            return f"{key} - the value is illegal.  Only true/false are perimited."
    elif typ == "list":
        if value is not None and "element" in ex:
            for el in (value if isinstance(value, list) else [value]):
                msg = check_item(key + "#dummy", el, grid)
                if msg != OK:
                    return msg
    elif typ == "map":
        if isinstance(value, dict):
            for k, v in value.items():
                msg = check_item(f"{key}#{k}", v, grid)
                if msg != OK:
                    return msg
    elif typ == "object":
        if isinstance(value, dict):
            for k, v in value.items():
                if f"{key}#{k}" in WAREHOUSE:
                    msg = check_item(f"{key}#{k}", v, grid)
                    if msg != OK:
                        return msg
    elif typ == "numberarray":
        if value is not None:
            for el in (value if isinstance(value, list) else [value]):
                if _num(el, float) is None:
                    return f"{key} - the value is not number format."
    return OK


def has_grid(mc) -> bool:
    params = (mc.train or {}).get("params") or {}
    return bool((mc.train or {}).get("gridConfigFile")) or any(
        isinstance(v, list) and k not in ("NumHiddenNodes", "ActivationFunc", "FixedLayers", "NumEmbedColumnIds")
        or (isinstance(v, list) and v and isinstance(v[0], list)) for k, v in params.items())


def validate_config(mc) -> list:
    """Every meta violation of the ModelConfig (empty list = valid)."""
    grid = has_grid(mc)
    causes = []
    groups = {"basic": mc.basic, "dataSet": mc.dataSet, "stats": mc.stats, "varSelect": mc.varSelect,
              "normalize": mc.normalize, "train": mc.train}
    for g, section in groups.items():
        items = section.d if hasattr(section, "d") else (section or {})
        for k, v in items.items():
            key = f"{g}#{k}"
            if key not in WAREHOUSE:          # unknown bean property: dropped by Jackson
                continue
            msg = check_item(key, v, grid)
            if msg != OK:
                causes.append(msg)
    for e in mc.evals or []:
        for k, v in (e.d if hasattr(e, "d") else e).items():
            key = f"evals#{k}"
            if key in WAREHOUSE:
                msg = check_item(key, v, grid)
                if msg != OK:
                    causes.append(msg)
    return causes
