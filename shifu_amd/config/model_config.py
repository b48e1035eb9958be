"""ModelConfig.json (C1): dict-backed sections with the reference's defaults.

Field names, enum spellings and defaults mirror ``J/container/obj/ModelBasicConf.java``,
``RawSourceData.java:40-112``, ``ModelSourceDataConf.java``, ``ModelStatsConf.java:34-95``,
``ModelVarSelectConf.java:36-123``, ``ModelNormalizeConf.java:33-92``,
``ModelTrainConf.java:43-191`` and ``EvalConfig.java:43-84``.  Sections keep unknown keys
(``@JsonIgnoreProperties(ignoreUnknown=true)``) and key order, so load -> save round-trips.

Vocabulary (SURVEY "trap"): ``is_binary`` == reference ``isRegression()`` (pos and neg
tags), ``is_multiclass`` == ``isClassification()``, ``is_linear_target`` == true regression.
"""
from __future__ import annotations

import copy
import getpass
import os
import time
from collections import OrderedDict

from . import jsonio
from .enums import (ALGORITHMS, BINNING_ALGORITHMS, BINNING_METHODS, MULTI_CLASSIFICATION, NORM_TYPES,
                    RUN_MODES, SOURCE_TYPES, parse_enum)

_MISSING = object()


class Section:
    DEFAULTS: "OrderedDict" = OrderedDict()
    # keys written by createInitModelConfig / a fresh Jackson serialization
    WRITE_KEYS: tuple = ()

    def __init__(self, d=None):
        self.d = OrderedDict(d) if d else OrderedDict()

    def __getattr__(self, k):
        if k == "d" or k.startswith("__"):
            raise AttributeError(k)
        d = self.__dict__.get("d")
        if d is not None and k in d:
            return d[k]
        if k in type(self).DEFAULTS:
            return copy.deepcopy(type(self).DEFAULTS[k])
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if k == "d":
            object.__setattr__(self, k, v)
        else:
            self.d[k] = v

    def __getitem__(self, k):
        return self.get(k)

    def copy_with(self, **overrides):
        c = type(self)(copy.deepcopy(self.d))
        c.d.update(overrides)
        return c

    def __setitem__(self, k, v):
        self.d[k] = v

    def __contains__(self, k):
        return k in self.d

    def get(self, k, default=None):
        if k in self.d and self.d[k] is not None:
            return self.d[k]
        if k in type(self).DEFAULTS and type(self).DEFAULTS[k] is not None:
            return copy.deepcopy(type(self).DEFAULTS[k])
        return default

    def to_dict(self, fill_defaults=False):
        out = OrderedDict()
        if fill_defaults:
            for k in self.WRITE_KEYS:
                out[k] = self.d.get(k, copy.deepcopy(self.DEFAULTS.get(k)))
        for k, v in self.d.items():
            out[k] = v.to_dict(fill_defaults) if isinstance(v, Section) else v
        return out


class BasicConf(Section):
    DEFAULTS = OrderedDict(name=None, author=None, description=None, version="0.13.0", runMode="LOCAL",
                           postTrainOn=False, customPaths=None)
    WRITE_KEYS = ("name", "author", "description", "version", "runMode", "postTrainOn", "customPaths")


class RawSourceData(Section):
    DEFAULTS = OrderedDict(source="LOCAL", dataPath=None, dataDelimiter="|", headerPath=None,
                           headerDelimiter="|", filterExpressions="", weightColumnName="",
                           targetColumnName=None, posTags=None, negTags=None, missingOrInvalidValues=["", "?"],
                           metaColumnNameFile=None, categoricalColumnNameFile=None, autoType=False,
                           autoTypeThreshold=0)
    WRITE_KEYS = ("source", "dataPath", "dataDelimiter", "headerPath", "headerDelimiter", "filterExpressions",
                  "weightColumnName", "targetColumnName", "posTags", "negTags", "missingOrInvalidValues",
                  "metaColumnNameFile", "categoricalColumnNameFile")


class DataSetConf(RawSourceData):
    DEFAULTS = OrderedDict(list(RawSourceData.DEFAULTS.items()) + [
        ("validationDataPath", None), ("validationFilterExpressions", ""), ("hybridColumnNameFile", None),
        ("segExpressionFile", None)])
    WRITE_KEYS = RawSourceData.WRITE_KEYS + ("validationDataPath", "validationFilterExpressions")


class StatsConf(Section):
    DEFAULTS = OrderedDict(maxNumBin=10, cateMaxNumBin=0, binningMethod="EqualPositive", sampleRate=1.0,
                           sampleNegOnly=False, numericalValueThreshold=1.7976931348623157e308,
                           binningAutoTypeEnable=False, binningAutoTypeThreshold=5, binningMergeEnable=True,
                           binningAlgorithm="SPDTI", psiColumnName="")
    WRITE_KEYS = ("maxNumBin", "cateMaxNumBin", "binningMethod", "sampleRate", "sampleNegOnly",
                  "binningAlgorithm", "psiColumnName")


class VarSelectConf(Section):
    DEFAULTS = OrderedDict(forceEnable=True, candidateColumnNameFile=None, forceSelectColumnNameFile=None,
                           forceRemoveColumnNameFile=None, filterEnable=True, filterNum=200, filterBy="KS",
                           filterOutRatio=0.05, autoFilterEnable=True, missingRateThreshold=0.98,
                           correlationThreshold=1.0, minIvThreshold=0.0, minKsThreshold=0.0,
                           postCorrelationMetric="IV", params=None)
    WRITE_KEYS = ("forceEnable", "candidateColumnNameFile", "forceSelectColumnNameFile",
                  "forceRemoveColumnNameFile", "filterEnable", "filterNum", "filterBy", "filterOutRatio",
                  "autoFilterEnable", "missingRateThreshold", "correlationThreshold", "minIvThreshold",
                  "minKsThreshold", "postCorrelationMetric", "params")


class NormalizeConf(Section):
    DEFAULTS = OrderedDict(stdDevCutOff=6.0, sampleRate=1.0, sampleNegOnly=False, normType="ZSCALE",
                           isParquet=False, correlation="None")
    WRITE_KEYS = ("stdDevCutOff", "sampleRate", "sampleNegOnly", "normType")


class TrainConf(Section):
    DEFAULTS = OrderedDict(baggingNum=1, baggingWithReplacement=False, baggingSampleRate=1.0, validSetRate=0.2,
                           sampleNegOnly=False, convergenceThreshold=0.0, numTrainEpochs=100,
                           epochsPerIteration=1, trainOnDisk=False, fixInitInput=False, stratifiedSample=False,
                           isContinuous=False, isCrossOver=False, workerThreadCount=4, numKFold=-1,
                           baggingSampleSeed=-1, upSampleWeight=1.0, algorithm="NN", params=None,
                           gridConfigFile=None, multiClassifyMethod="NATIVE", customPaths=None)
    WRITE_KEYS = ("baggingNum", "baggingWithReplacement", "baggingSampleRate", "validSetRate",
                  "numTrainEpochs", "isContinuous", "workerThreadCount", "algorithm", "params",
                  "customPaths")


class EvalConf(Section):
    DEFAULTS = OrderedDict(name=None, dataSet=None, performanceBucketNum=10, performanceScoreSelector="mean",
                           scoreMetaColumnNameFile=None, customPaths=None, scoreScale=1000, normAllColumns=False,
                           gbtConvertToProb=True, gbtScoreConvertStrategy="OLD_SIGMOID")
    WRITE_KEYS = ("name", "dataSet", "performanceBucketNum", "performanceScoreSelector",
                  "scoreMetaColumnNameFile", "customPaths")

    def __init__(self, d=None):
        super().__init__(d)
        ds = self.d.get("dataSet")
        if ds is not None and not isinstance(ds, Section):
            self.d["dataSet"] = RawSourceData(ds)


# ---------------------------------------------------------------------------------------------
# default algorithm params (ModelTrainConf.createParamsByAlg J/container/obj/ModelTrainConf.java:531-612)
# ---------------------------------------------------------------------------------------------
def create_params_by_alg(alg: str) -> "OrderedDict":
    alg = alg.upper()
    p = OrderedDict()
    if alg == "NN":
        p.update(Propagation="R", LearningRate=0.1, NumHiddenLayers=1, NumHiddenNodes=[50],
                 ActivationFunc=["tanh"], RegularizedConstant=0.0)
    elif alg == "SVM":
        p.update(Kernel="linear", Gamma=1.0, Const=1.0)
    elif alg == "RF":
        p.update(TreeNum="10", FeatureSubsetStrategy="TWOTHIRDS", MaxDepth=10, MinInstancesPerNode=1,
                 MinInfoGain=0.0, Impurity="variance", Loss="squared")
    elif alg == "GBT":
        p.update(TreeNum="100", FeatureSubsetStrategy="TWOTHIRDS", MaxDepth=7, MinInstancesPerNode=5,
                 MinInfoGain=0.0, DropoutRate=0.0, Impurity="variance", LearningRate=0.05, Loss="squared")
    elif alg == "LR":
        p.update(Propagation="R", LearningRate=0.1, RegularizedConstant=0.0, L1orL2="NONE")
    elif alg == "TENSORFLOW":
        p.update(LearningRate=0.1, NumHiddenLayers=1, NumHiddenNodes=[50], ActivationFunc=["relu"],
                 **{"TF.alg": "DNN", "CheckpointInterval": 0, "TF.optimizer": "Adam", "TF.loss": "entropy"})
    elif alg == "WDL":
        p.update(LearningRate=0.1, NumEmbedColumnIds=[], NumHiddenLayers=1, NumHiddenNodes=[50],
                 ActivationFunc=["relu"], WDLL2Reg=1e-8, EmbedOutputs=8)
    return p


class ModelConfig:
    SECTIONS = (("basic", BasicConf), ("dataSet", DataSetConf), ("stats", StatsConf),
                ("varSelect", VarSelectConf), ("normalize", NormalizeConf), ("train", TrainConf))

    def __init__(self, d=None, path: str | None = None):
        d = OrderedDict(d or {})
        self.extra = OrderedDict()
        for k, cls in self.SECTIONS:
            setattr(self, k, cls(d.pop(k, None)))
        self.evals = [EvalConf(e) for e in (d.pop("evals", None) or [])]
        self.extra.update(d)
        self.path = path

    # ---- IO ------------------------------------------------------------------------------
    @staticmethod
    def load(path: str) -> "ModelConfig":
        return ModelConfig(jsonio.load(path), path=os.path.abspath(path))

    def to_dict(self, fill_defaults=False):
        out = OrderedDict()
        for k, _ in self.SECTIONS:
            out[k] = getattr(self, k).to_dict(fill_defaults)
        out["evals"] = [e.to_dict(fill_defaults) for e in self.evals]
        out.update(self.extra)
        return out

    def save(self, path: str | None = None):
        path = path or self.path
        jsonio.dump(self.to_dict(), path)
        self.path = os.path.abspath(path)

    def copy(self) -> "ModelConfig":
        return ModelConfig(jsonio.loads(jsonio.dumps(self.to_dict())), self.path)

    @property
    def model_set_dir(self) -> str:
        return os.path.dirname(self.path) if self.path else os.getcwd()

    def resolve(self, p: str | None) -> str | None:
        """Resolve a path in the config relative to the model-set directory."""
        if p is None or p == "":
            return p
        if os.path.isabs(p):
            return p
        cand = os.path.normpath(os.path.join(self.model_set_dir, p))
        if os.path.exists(cand) or not os.path.exists(p):
            return cand
        return os.path.abspath(p)

    # ---- helpers mirroring ModelConfig.java --------------------------------------------------
    @property
    def name(self):
        return self.basic.get("name")

    @property
    def algorithm(self) -> str:
        return parse_enum(self.train.get("algorithm", "NN"), ALGORITHMS)

    @property
    def run_mode(self) -> str:
        return parse_enum(self.basic.get("runMode", "LOCAL"), RUN_MODES)

    @property
    def pos_tags(self):
        return list(self.dataSet.get("posTags") or [])

    @property
    def neg_tags(self):
        return list(self.dataSet.get("negTags") or [])

    def is_binary(self) -> bool:          # reference isRegression()
        return bool(self.pos_tags) and bool(self.neg_tags)

    def is_multiclass(self) -> bool:      # reference isClassification()
        return bool(self.pos_tags) != bool(self.neg_tags)

    def is_linear_target(self) -> bool:   # CommonUtils.isLinearTarget: no tags, numeric target
        return not self.pos_tags and not self.neg_tags

    def tags(self):
        """Class tags: binary -> [pos..., neg...]; multi-class -> the non-empty tag list."""
        if self.is_binary():
            return self.pos_tags + self.neg_tags
        return self.pos_tags or self.neg_tags

    def flatten_tags(self):
        out = []
        for t in self.tags():
            out.extend([x for x in str(t).split("|") if x.strip()] if "|" in str(t) else [t])
        return out

    def set_tags(self):
        return [set(x for x in str(t).split("|") if x.strip()) if "|" in str(t) else {t} for t in self.tags()]

    @property
    def params(self):
        p = self.train.get("params")
        if p is None:
            p = create_params_by_alg(self.algorithm)
            self.train.params = p
        return p

    def param(self, key, default=None):
        p = self.params or {}
        for k, v in p.items():
            if k.lower() == key.lower():
                return v
        return default

    @property
    def norm_type(self) -> str:
        return parse_enum(self.normalize.get("normType", "ZSCALE"), NORM_TYPES)

    @property
    def binning_method(self) -> str:
        return parse_enum(self.stats.get("binningMethod", "EqualPositive"), BINNING_METHODS)

    @property
    def binning_algorithm(self) -> str:
        return parse_enum(self.stats.get("binningAlgorithm", "SPDTI"), BINNING_ALGORITHMS)

    @property
    def multi_classify_method(self) -> str:
        return parse_enum(self.train.get("multiClassifyMethod", "NATIVE"), MULTI_CLASSIFICATION)

    def is_one_vs_all(self) -> bool:
        return self.multi_classify_method in ("ONEVSALL", "ONEVSREST")

    @property
    def source_type(self) -> str:
        return parse_enum(self.dataSet.get("source", "LOCAL"), SOURCE_TYPES)

    @property
    def bagging_num(self) -> int:
        return int(self.train.get("baggingNum", 1))

    @property
    def num_epochs(self) -> int:
        return int(self.train.get("numTrainEpochs", 100))

    @property
    def missing_values(self):
        v = self.dataSet.get("missingOrInvalidValues")
        return list(v) if v is not None else ["", "?"]

    def eval_by_name(self, name: str):
        for e in self.evals:
            if (e.get("name") or "").lower() == name.lower():
                return e
        return None

    def _read_names(self, key_or_path, section=None):
        from ..data.reader import read_column_name_file
        p = key_or_path
        if section is not None:
            p = section.get(key_or_path)
        if not p:
            return []
        return read_column_name_file(self.resolve(p))

    def meta_column_names(self):
        return self._read_names("metaColumnNameFile", self.dataSet)

    def categorical_column_names(self):
        return self._read_names("categoricalColumnNameFile", self.dataSet)

    def force_select_names(self):
        return self._read_names("forceSelectColumnNameFile", self.varSelect)

    def force_remove_names(self):
        return self._read_names("forceRemoveColumnNameFile", self.varSelect)

    def candidate_names(self):
        return self._read_names("candidateColumnNameFile", self.varSelect)

    def hybrid_column_names(self) -> dict:
        """hybrid column file lines: ``name`` or ``name<TAB/,>threshold`` (ModelConfig.java:700-737)."""
        p = self.dataSet.get("hybridColumnNameFile")
        out = {}
        if not p:
            return out
        path = self.resolve(p)
        if not os.path.exists(path):
            return out
        for line in open(path, encoding="utf-8"):
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            parts = [x for x in line.replace("\t", ",").split(",") if x.strip()]
            out[parts[0].strip()] = float(parts[1]) if len(parts) > 1 else 1.7976931348623157e308
        return out

    def segment_filter_expressions(self):
        p = self.dataSet.get("segExpressionFile")
        if not p:
            return []
        path = self.resolve(p)
        if not os.path.exists(path):
            return []
        return [l.strip() for l in open(path, encoding="utf-8") if l.strip() and not l.startswith("#")]


def create_init_model_config(name: str, alg: str = "NN", description: str | None = None,
                             shifu_home: str | None = None) -> ModelConfig:
    """``ModelConfig.createInitModelConfig`` (J/container/obj/ModelConfig.java:168-328)."""
    alg = parse_enum(alg, ALGORITHMS)
    home = shifu_home or os.environ.get("SHIFU_HOME", os.getcwd())
    ds = os.path.join(home, "example", "cancer-judgement", "DataStore", "DataSet1")
    es = os.path.join(home, "example", "cancer-judgement", "DataStore", "EvalSet1")
    try:
        user = getpass.getuser()
    except Exception:   # pragma: no cover
        user = "shifu"
    d = OrderedDict()
    d["basic"] = OrderedDict(name=name, author=user,
                             description=description or "Created at " + time.strftime("%Y-%m-%d %H:%M:%S"),
                             version="0.13.0", runMode="LOCAL", postTrainOn=False, customPaths=OrderedDict())
    d["dataSet"] = OrderedDict(source="LOCAL", dataPath=ds, dataDelimiter="|", headerPath=os.path.join(ds, ".pig_header"),
                               headerDelimiter="|", filterExpressions="", weightColumnName="",
                               targetColumnName="diagnosis", posTags=["M"], negTags=["B"],
                               missingOrInvalidValues=["", "*", "#", "?", "null", "~"],
                               metaColumnNameFile="columns/meta.column.names",
                               categoricalColumnNameFile="columns/categorical.column.names",
                               validationDataPath=None, validationFilterExpressions="")
    d["stats"] = OrderedDict(maxNumBin=10, cateMaxNumBin=0, binningMethod="EqualPositive", sampleRate=1.0,
                             sampleNegOnly=False, binningAlgorithm="SPDTI", psiColumnName="")
    d["varSelect"] = OrderedDict(forceEnable=True, candidateColumnNameFile=None,
                                 forceSelectColumnNameFile="columns/forceselect.column.names",
                                 forceRemoveColumnNameFile="columns/forceremove.column.names",
                                 filterEnable=True, filterNum=200, filterBy="KS", filterOutRatio=0.05,
                                 autoFilterEnable=True, missingRateThreshold=0.98, correlationThreshold=1.0,
                                 minIvThreshold=0.0, minKsThreshold=0.0, postCorrelationMetric="IV",
                                 params=None)
    # WDL trains on z-scored numerics + category indices (the reference pairs WDL with ZSCALE_INDEX,
    # TrainModelProcessor.java:587; WDLWorker reads a category index per categorical input)
    d["normalize"] = OrderedDict(stdDevCutOff=6.0, sampleRate=1.0, sampleNegOnly=False,
                                 normType="ZSCALE_INDEX" if alg == "WDL" else "ZSCALE")
    epochs = {"NN": 200, "SVM": 100, "RF": 20000, "GBT": 20000, "LR": 100, "TENSORFLOW": 100}.get(alg, 100)
    d["train"] = OrderedDict(baggingNum=5, baggingWithReplacement=False, baggingSampleRate=1.0, validSetRate=0.2,
                             numTrainEpochs=epochs, isContinuous=False, workerThreadCount=4, algorithm=alg,
                             params=create_params_by_alg(alg), customPaths=OrderedDict())
    ev = OrderedDict(name="Eval1", dataSet=OrderedDict(
        source="LOCAL", dataPath=es, dataDelimiter="|", headerPath=os.path.join(es, ".pig_header"),
        headerDelimiter="|", filterExpressions="", weightColumnName="", targetColumnName="diagnosis",
        posTags=["M"], negTags=["B"], missingOrInvalidValues=["", "*", "#", "?", "null", "~"],
        metaColumnNameFile="columns/Eval1.meta.column.names"),
        performanceBucketNum=10, performanceScoreSelector="mean",
        scoreMetaColumnNameFile="columns/Eval1score.meta.column.names", customPaths=OrderedDict())
    d["evals"] = [ev]
    return ModelConfig(d)
