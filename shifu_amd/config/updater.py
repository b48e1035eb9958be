"""Column flag updater (C5) and namespaced column names (C6).

``BasicUpdater.updateColumnConfig`` (J/util/updater/BasicUpdater.java:94-150): target / meta /
forceRemove / forceSelect / weight / candidate flags and N/C/H types, re-applied at every step
so that edits of the column-name files take effect.  ``NSColumn`` (J/column/NSColumn.java):
``ns::name`` names compare on the simple name unless ``shifu.namespace.strict.mode``.
"""
from __future__ import annotations

from . import environment as env


def simple_name(name: str) -> str:
    if name is None:
        return ""
    n = str(name).strip()
    return n.rsplit("::", 1)[-1] if "::" in n else n


def ns_equal(a, b) -> bool:
    if a is None or b is None:
        return False
    if env.get_bool("shifu.namespace.strict.mode", False):
        return str(a).strip() == str(b).strip()
    return simple_name(a) == simple_name(b)


class NSSet:
    def __init__(self, names):
        self.strict = env.get_bool("shifu.namespace.strict.mode", False)
        self.s = {self._k(n) for n in (names or []) if n is not None and str(n).strip()}

    def _k(self, n):
        return str(n).strip() if self.strict else simple_name(n)

    def __contains__(self, n):
        return self._k(n) in self.s

    def __len__(self):
        return len(self.s)


def update_column_flags(mc, ccs, step: str = "INIT"):
    """Re-derive flags/types of every column from ModelConfig + the column name files."""
    target = mc.dataSet.get("targetColumnName")
    weight = mc.dataSet.get("weightColumnName") or None
    meta = NSSet(mc.meta_column_names())
    force_remove = NSSet(mc.force_remove_names() if mc.varSelect.get("forceEnable", True) else [])
    force_select = NSSet(mc.force_select_names() if mc.varSelect.get("forceEnable", True) else [])
    candidates = NSSet(mc.candidate_names())
    cats = NSSet(mc.categorical_column_names())
    hybrid = mc.hybrid_column_names()
    hyb = NSSet(list(hybrid.keys()))
    has_tags = bool(mc.tags())
    segs = mc.segment_filter_expressions()
    raw_names = {c.name for c in ccs[: len(ccs) // (len(segs) + 1)]} if segs else set()
    for c in ccs:
        name = c.name
        keep_type = c.type
        if segs:                    # segment copy "<col>_<k>": flags/type follow the base column
            from ..data.segments import split_name
            base, k = split_name(name, len(segs), raw_names)
            if k:
                c.flag = None
                if ns_equal(target, base) or (weight and ns_equal(weight, base)):
                    c.flag = "ForceRemove"          # VarSelectModelProcessor :157-176 (shadow targets)
                elif base in meta:
                    c.flag = "Meta"
                elif base in force_remove:
                    c.flag = "ForceRemove"
                c.type = "C" if base in cats else ("H" if base in hyb else "N")
                if c.is_meta() or c.is_force_remove():
                    c.final_select = False
                continue
        c.flag = None
        if ns_equal(target, name):
            c.flag = "Target"
        elif name in meta:
            c.flag = "Meta"
        elif name in force_remove:
            c.flag = "ForceRemove"
        elif name in force_select:
            if len(candidates) == 0 or name in candidates:
                c.flag = "ForceSelect"
        elif weight and ns_equal(weight, name):
            c.flag = "Weight"
        elif name in candidates:
            c.flag = "Candidate"
        if weight and ns_equal(weight, name):
            c.type = "N"
        elif ns_equal(target, name):
            c.type = "C" if has_tags else "N"
        elif name in hyb:
            c.type = "H"
            c.d["hybridThreshold"] = hybrid.get(simple_name(name), hybrid.get(name))
        elif name in cats:
            c.type = "C"
        elif step in ("INIT",) or keep_type is None:
            c.type = "N"
        elif keep_type == "C" and step != "INIT":
            c.type = "C"       # keep auto-typed categorical columns after init
        else:
            c.type = "N" if keep_type not in ("N", "C", "H") else keep_type
        if c.is_target() or c.is_meta() or c.is_force_remove() or c.is_weight():
            c.final_select = False
        if step in ("VARSELECT", "TRAIN") and c.is_force_select():
            c.final_select = True
    return ccs
