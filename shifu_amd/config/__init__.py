"""L2 config & metadata: ModelConfig / ColumnConfig (same JSON as the reference), enums,
layered flags, column flag updater, validation, on-disk layout."""
from .model_config import ModelConfig, create_init_model_config, create_params_by_alg
from .column_config import (ColumnConfig, load_column_configs, save_column_configs, selected_columns,
                            target_column, weight_column, has_candidates)
from .path_finder import PathFinder
from . import environment, jsonio, enums, validator, updater, errors

__all__ = ["ModelConfig", "create_init_model_config", "create_params_by_alg", "ColumnConfig",
           "load_column_configs", "save_column_configs", "selected_columns", "target_column",
           "weight_column", "has_candidates", "PathFinder", "environment", "jsonio", "enums",
           "validator", "updater", "errors"]
