"""L5 model artifact formats: Encog EG / binary .nn, .gbt/.rf v4, .lr, .wdl, PMML."""
