"""Programmatic Step API (A5): ``Step.process()`` objects over an in-memory ModelConfig /
ColumnConfig list, mirroring ``ml/shifu/common/Step.java:30-80`` and the ``InitStep`` /
``StatsStep`` / ``NormStep`` / ``VarSelStep`` / ``TrainStep`` / ``EvalStep`` classes
(``train/TrainStep.java:30-67``).  Each step persists to the model-set directory exactly like
the CLI verb and returns the updated ColumnConfig list, so steps chain in-process::

    ms = ModelSet("/path/to/modelset")
    ccs = InitStep(ms).process()
    ccs = StatsStep(ms).process()
    ccs = VarSelStep(ms).process()
    NormStep(ms).process()
    TrainStep(ms).process()
    EvalStep(ms).process()
"""
from __future__ import annotations

from .base import ModelSet


class Step:
    """Base: holds the model set; ``process()`` runs the step and returns the ColumnConfig list."""
    name = "step"

    def __init__(self, ms: ModelSet | str, **options):
        self.ms = ms if isinstance(ms, ModelSet) else ModelSet(ms)
        self.options = options

    @property
    def root(self):
        return self.ms.root

    def _reload(self):
        fresh = ModelSet(self.root)
        self.ms.mc, self.ms.ccs = fresh.mc, fresh.ccs
        return self.ms.ccs

    def process(self):
        self.run()
        return self._reload()

    def run(self):   # pragma: no cover - abstract
        raise NotImplementedError


class CreateStep(Step):
    name = "new"

    def __init__(self, parent: str, model_name: str, alg: str = "NN", description: str | None = None):
        from .create import create_model_set
        self.root_path = create_model_set(model_name, alg, description, parent)
        super().__init__(self.root_path)

    def run(self):
        return 0


class InitStep(Step):
    name = "init"

    def run(self):
        from .create import run_init
        return run_init(self.root, self.options.get("auto_type"))


class StatsStep(Step):
    name = "stats"

    def run(self):
        from .stats import run_stats
        o = self.options
        return run_stats(self.root, o.get("correlation", False), o.get("psi", False), o.get("rebin", False),
                         o.get("expected_bins"), o.get("iv_keep_ratio", 1.0))


class NormStep(Step):
    name = "norm"

    def run(self):
        from .norm import run_norm
        return run_norm(self.root, shuffle=self.options.get("shuffle", False))


class VarSelStep(Step):
    name = "varsel"

    def run(self):
        from .varsel import run_varsel
        o = self.options
        return run_varsel(self.root, o.get("reset", False), False, o.get("autofilter", False),
                          o.get("recover", False), o.get("recursive", 1))


class TrainStep(Step):
    name = "train"

    def run(self):
        from .train import TrainStep as _Train
        return _Train(self.ms, dry=self.options.get("dry", False), device=self.options.get("device")).process()


class PostTrainStep(Step):
    name = "posttrain"

    def run(self):
        from .posttrain import run_posttrain
        return run_posttrain(self.root)


class EvalStep(Step):
    name = "eval"

    def run(self):
        from .evaluate import run_eval
        return run_eval(self.root, self.options.get("action", "run"), self.options.get("eval_name"))


class ExportStep(Step):
    name = "export"

    def run(self):
        from .export import run_export
        return run_export(self.root, self.options.get("type", "pmml"))


PIPELINE = (InitStep, StatsStep, VarSelStep, NormStep, TrainStep, EvalStep)


def run_pipeline(root: str, steps=PIPELINE, **options):
    """Run the standard pipeline in-process (A4 regression driver equivalent)."""
    ms = ModelSet(root)
    for cls in steps:
        cls(ms, **options.get(cls.name, {})).process()
    return ms
