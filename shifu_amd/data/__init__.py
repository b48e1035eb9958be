"""L1 data: delimited reader (native C++ parser), JEXL-subset expressions, purify/tag/sample/
weight, columnar caches and synthetic generators."""
from .reader import RawTable, Column, read_table, read_header, read_column_name_file, list_data_files
from .purifier import ModelData, purify, load_dataset
from .expr import Evaluator, compile_expr

__all__ = ["RawTable", "Column", "read_table", "read_header", "read_column_name_file", "list_data_files",
           "ModelData", "purify", "load_dataset", "Evaluator", "compile_expr"]
