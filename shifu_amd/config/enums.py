"""Enums of the config schema (case-insensitive parsing like the reference ``*Deserializer``s)."""
from __future__ import annotations

RUN_MODES = ("LOCAL", "DIST", "MAPRED")
SOURCE_TYPES = ("LOCAL", "HDFS", "S3")
BINNING_METHODS = ("EqualNegtive", "EqualInterval", "EqualPositive", "EqualTotal", "WeightEqualNegative",
                   "WeightEqualInterval", "WeightEqualPositive", "WeightEqualTotal")
BINNING_ALGORITHMS = ("Native", "SPDT", "SPDTI", "MunroPat", "MunroPatI", "DynamicBinning")
NORM_TYPES = ("OLD_ZSCORE", "OLD_ZSCALE", "ZSCORE", "ZSCALE", "WOE", "WEIGHT_WOE", "HYBRID", "WEIGHT_HYBRID",
              "WOE_ZSCORE", "WOE_ZSCALE", "WEIGHT_WOE_ZSCORE", "WEIGHT_WOE_ZSCALE", "ONEHOT", "ZSCALE_ONEHOT",
              "ASIS_WOE", "ASIS_PR", "DISCRETE_ZSCORE", "DISCRETE_ZSCALE", "ZSCALE_INDEX", "ZSCORE_INDEX",
              "WOE_INDEX", "WOE_ZSCALE_INDEX")
ALGORITHMS = ("NN", "LR", "SVM", "DT", "RF", "GBT", "TENSORFLOW", "WDL", "GENERIC")
MULTI_CLASSIFICATION = ("NATIVE", "ONEVSALL", "ONEVSREST", "ONEVSONE")
POST_CORRELATION_METRICS = ("IV", "KS", "SE")
COLUMN_FLAGS = ("ForceSelect", "ForceRemove", "Candidate", "Meta", "Target", "Weight")
COLUMN_TYPES = ("A", "N", "C", "H")


def parse_enum(value, choices, default=None):
    if value is None:
        return default if default is not None else choices[0]
    s = str(value).strip()
    for c in choices:
        if c.lower() == s.lower():
            return c
    if default is not None:
        return default
    raise ValueError(f"{value!r} is not one of {choices}")


def is_woe_norm(nt: str) -> bool:
    return nt in ("WOE", "WEIGHT_WOE", "WOE_ZSCORE", "WOE_ZSCALE", "WEIGHT_WOE_ZSCORE", "WEIGHT_WOE_ZSCALE")


def is_index_norm(nt: str) -> bool:
    return nt in ("ZSCALE_INDEX", "ZSCORE_INDEX", "WOE_INDEX", "WOE_ZSCALE_INDEX")
