"""L4 algorithms: binning, column stats/KS/IV/WOE, correlation, PSI, normalization, variable
selection, evaluation metrics, post-train, early stop, grid search."""
