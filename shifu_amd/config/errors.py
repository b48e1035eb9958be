"""Error codes (C7) - ``J/exception/ShifuErrorCode.java`` / ``ShifuException``."""
from __future__ import annotations

from enum import Enum


class ShifuErrorCode(Enum):
    ERROR_MODELCONFIG_NOT_VALIDATION = (1001, "The ModelConfig.json is not valid.")
    ERROR_COLUMNCONFIG_NOT_FOUND = (1002, "ColumnConfig.json is not found, run `shifu init` first.")
    ERROR_MODEL_FILE_NOT_FOUND = (1003, "Model file is not found, run `shifu train` first.")
    ERROR_NO_TARGET_COLUMN = (1004, "No target column is found.")
    ERROR_MODELSET_NOT_FOUND = (1005, "Model set is not found.")
    ERROR_INPUT_NOT_FOUND = (1006, "Input data is not found.")
    ERROR_HEADER_NOT_FOUND = (1007, "Header file is not found or empty.")
    ERROR_UNSUPPORT_MODE = (1008, "Unsupported mode.")
    ERROR_UNSUPPORT_ALG = (1009, "Unsupported algorithm.")
    ERROR_EVALCONFIG_NOT_FOUND = (1010, "Eval set is not found.")
    ERROR_MODEL_EVALSET_ALREADY_EXIST = (1011, "Eval set already exists.")
    ERROR_INVALID_FILTER_EXPRESSION = (1012, "Filter expression is invalid.")
    ERROR_NO_SELECTED_COLUMN = (1013, "No selected column; run varsel or check ColumnConfig.json.")
    ERROR_INVALID_MODEL = (1014, "Model file is invalid or corrupted.")
    ERROR_EXPORT_TYPE = (1015, "Unsupported export type.")
    ERROR_GRID_SEARCH_FILE_CONFIG = (1016, "Grid search config file is invalid.")
    ERROR_SHIFU_CONFIG = (1017, "shifuconfig error.")
    ERROR_MODELCONFIG_NOT_EXIST = (1018, "ModelConfig.json does not exist; run `shifu new` or cd into the model set.")
    ERROR_EVALSCORE = (1019, "No eval score is generated.")
    ERROR_EVALCONFMTR = (1020, "Confusion matrix is empty.")

    @property
    def code(self):
        return self.value[0]

    @property
    def message(self):
        return self.value[1]


class ShifuException(RuntimeError):
    def __init__(self, err: ShifuErrorCode, detail: str = ""):
        super().__init__(f"[{err.code}] {err.message}" + (f" {detail}" if detail else ""))
        self.err = err
