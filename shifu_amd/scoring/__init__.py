"""Scoring runtime: model loading, NN/LR/tree scorers, independent models."""
