"""Model engines: NN (MLP), LR, GBT/RF trees, WDL."""
