"""On-disk model-set layout (D1), names from ``J/util/Constants.java:25-192`` and the getters of
``J/fs/PathFinder.java:152-1080``.  Everything is local FS (the HDFS mirror of the reference is
replaced by node-local NVMe / shared FS; ``customPaths`` overrides are honoured)."""
from __future__ import annotations

import os

MODELS = "models"
MODELS_TMP = "modelsTmp"
TMP = "tmp"
VAR_SEL = "varsel"
EVAL_DIR = "evals"
COLUMN_DIR = "columns"
MODEL_CONFIG = "ModelConfig.json"
COLUMN_CONFIG = "ColumnConfig.json"
COMBO_CONFIG = "ComboTrain.json"
COLUMN_STATS_CSV = "ColumnStats.csv"
HEAD = ".HEAD"


class PathFinder:
    def __init__(self, model_config, root: str | None = None):
        self.mc = model_config
        self.root = os.path.abspath(root or model_config.model_set_dir)

    def _custom(self, key, section=None):
        cp = (section or self.mc.basic).get("customPaths") or {}
        v = cp.get(key) if isinstance(cp, dict) else None
        return v or None

    def p(self, *parts) -> str:
        return os.path.join(self.root, *parts)

    # configs ------------------------------------------------------------------------------
    @property
    def model_config(self):
        return self.p(MODEL_CONFIG)

    @property
    def column_config(self):
        return self.p(COLUMN_CONFIG)

    @property
    def column_dir(self):
        return self.p(COLUMN_DIR)

    # data artifacts (replace Pig/MR output folders; columnar binary caches) ---------------------
    @property
    def tmp_dir(self):
        return self.p(TMP)

    @property
    def pre_training_stats(self):
        return self._custom("preTrainStatsPath") or self.p(TMP, "PreTrainingStats")

    @property
    def stats_small_bins(self):
        return self.p(TMP, "StatsSmallBins")

    @property
    def binning_info(self):
        return self.p(TMP, "binning_info.txt")

    @property
    def auto_type_path(self):
        return self._custom("autoTypePath") or self.p(TMP, "AutoTypePath")

    @property
    def correlation_path(self):
        return self._custom("correlationPath") or self.p(TMP, "CorrelationPath")

    @property
    def correlation_csv(self):
        return self.p("correlation.csv")

    @property
    def normalized_data(self):
        return self._custom("normalizedDataPath") or self.p(TMP, "NormalizedData")

    @property
    def normalized_validation_data(self):
        return self._custom("normalizedValidationDataPath") or self.p(TMP, "NormalizedValidationData")

    @property
    def selected_raw_data(self):
        """tmp/SelectedRawData (customPaths.selectedRawDataPath), PathFinder.getSelectedRawDataPath :323."""
        return self._custom("selectedRawDataPath") or self.p(TMP, "SelectedRawData")

    @property
    def cleaned_data(self):
        return self._custom("cleanedDataPath") or self.p(TMP, "CleanedData")

    @property
    def cleaned_validation_data(self):
        return self._custom("cleanedValidationDataPath") or self.p(TMP, "CleanedValidationData")

    @property
    def shuffled_data(self):
        return self.p(TMP, "ShuffledData")

    @property
    def train_scores(self):
        return self._custom("trainScoresPath") or self.p(TMP, "TrainScores")

    @property
    def bin_avg_score(self):
        return self._custom("binAvgScorePath") or self.p(TMP, "BinAvgScore")

    @property
    def psi_path(self):
        return self._custom("StatsPSIPath") or self.p(TMP, "PSI")

    @property
    def encoded_train_data(self):
        return self.p(TMP, "encodedTrainData")

    def encoded_eval_data(self, name):
        return self.p(TMP, "encodedEval" + name)

    # models -------------------------------------------------------------------------------
    @property
    def models_dir(self):
        return self._custom("modelsPath", self.mc.train) or self.p(MODELS)

    @property
    def bmodels_dir(self):
        """Binary v1 ``.nn`` copies (PathFinder.getNNBinaryModelsPath :521)."""
        return self.p("bmodels")

    @property
    def valerr_dir(self):
        return self.p(TMP, "valerr")

    @property
    def tmp_models_dir(self):
        return self.p(MODELS_TMP)

    def model_path(self, i: int, ext: str) -> str:
        """``models/model{i}.{ext}`` (TrainModelProcessor.getModelName :1807-1810)."""
        return os.path.join(self.models_dir, f"model{i}.{ext.lower().lstrip('.')}")

    def tmp_model_path(self, trainer: int, it: int, ext: str) -> str:
        return os.path.join(self.tmp_models_dir, f"model{trainer}-{it}.{ext.lower()}")

    @property
    def checkpoint_dir(self):
        return self.p(TMP, "checkpoints")

    @property
    def progress_log(self):
        return self.p(TMP, "train.progress.log")

    @property
    def metrics_jsonl(self):
        return self.p(TMP, "metrics.jsonl")

    @property
    def feature_importance(self):
        return self.p(MODELS, "feature.importance")

    # varsel -------------------------------------------------------------------------------
    @property
    def varsel_dir(self):
        return self.p(VAR_SEL)

    @property
    def varsel_history(self):
        return self.p(VAR_SEL, "varsel.history")

    def varsel_cc_backup(self, n: int):
        return self.p(VAR_SEL, f"ColumnConfig.json.{n}")

    def varsel_se(self, n: int):
        return self.p(VAR_SEL, f"se.{n}")

    # eval ---------------------------------------------------------------------------------
    def eval_dir(self, name):
        return self.p(EVAL_DIR, name)

    def eval_score(self, ev):
        return self._custom("scorePath", ev) or os.path.join(self.eval_dir(ev.get("name")), "EvalScore")

    def eval_performance(self, ev):
        return self._custom("performancePath", ev) or os.path.join(self.eval_dir(ev.get("name")),
                                                                     "EvalPerformance.json")

    def eval_confusion_matrix(self, ev):
        return self._custom("confusionMatrixPath", ev) or os.path.join(self.eval_dir(ev.get("name")),
                                                                         "EvalConfusionMatrix")

    def eval_normalized(self, ev):
        return os.path.join(self.eval_dir(ev.get("name")), "EvalNormalized")

    def eval_meta_score(self, ev):
        return os.path.join(self.eval_dir(ev.get("name")), "EvalMetaScore")

    def eval_models_dir(self, ev):
        return self._custom("modelsPath", ev) or self.models_dir

    # misc ---------------------------------------------------------------------------------
    @property
    def head_file(self):
        return self.p(HEAD)

    def backup_column_config(self, ts: str):
        return self.p(TMP, f"ColumnConfig.json.{ts}")

    @property
    def column_stats_csv(self):
        return self.p(COLUMN_STATS_CSV)

    @property
    def combo_config(self):
        return self.p(COMBO_CONFIG)

    @property
    def reason_code_map(self):
        return self.p("ReasonCodeMap.json")

    def ensure(self, path: str) -> str:
        os.makedirs(path if not os.path.splitext(path)[1] else os.path.dirname(path), exist_ok=True)
        return path
