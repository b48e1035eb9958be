"""A small PMML 4.2 evaluator for the subset ``formats/pmml.py`` exports (I7 verification).

The reference checks exported PMML against its own scores with a PMML engine
(``PMMLVerifySuit`` T/.../PMMLVerifySuit.java:121-190: evaluate every record of the eval set with
the PMML, compare with the ``shifu eval`` score within a tolerance).  No PMML engine is installed
here, so this module implements the elements the exporter writes, from the PMML 4.2 semantics:

* DataDictionary (categorical ``Value`` lists define the valid values), MiningSchema
  (``missingValueReplacement``, ``invalidValueTreatment="asMissing"``);
* LocalTransformations ``DerivedField``: ``NormContinuous`` (piecewise-linear ``LinearNorm``,
  ``outliers="asExtremeValues"``, ``mapMissingTo``), ``MapValues`` + ``InlineTable``
  (``mapMissingTo`` / ``defaultValue``), ``Discretize`` (closedOpen ``Interval`` bins), ``FieldRef``;
* NeuralNetwork (NeuralInputs, NeuralLayer with per-layer ``activationFunction``, Neuron bias +
  Con weights, NeuralOutputs), RegressionModel (NumericPredictor, intercept,
  ``normalizationMethod`` logit/none), TreeModel (Node, first-true-child, ``score``), MiningModel
  ``Segmentation`` (sum / weightedSum / average / weightedAverage); ``Constant`` / ``Apply``
  expressions and the ``Output`` element (predictedValue / transformedValue) of reference-written
  PMML (``src/test/resources/dttest/model/golf0*.pmml``).
Records are dicts {field name: raw value (str / float / None)}.
"""
from __future__ import annotations

import math
import shlex
import xml.etree.ElementTree as ET

import numpy as np

_ACT = {
    "logistic": lambda z: 1.0 / (1.0 + math.exp(-z)) if z > -700 else 0.0,
    "tanh": math.tanh, "identity": lambda z: z, "rectifier": lambda z: max(0.0, z), "sine": math.sin,
    "exponential": math.exp, "threshold": lambda z: 1.0 if z > 0 else 0.0,
}


def _strip(tag: str) -> str:
    return tag.split("}", 1)[1] if "}" in tag else tag


def _kids(el, name):
    return [c for c in el if _strip(c.tag) == name]


def _kid(el, name):
    k = _kids(el, name)
    return k[0] if k else None


def _num(v):
    if v is None:
        return None
    try:
        f = float(v)
    except (TypeError, ValueError):
        return None
    return None if f != f else f


class PMMLModel:
    def __init__(self, path_or_xml: str):
        text = open(path_or_xml, encoding="utf-8").read() if not path_or_xml.lstrip().startswith("<") \
            else path_or_xml
        self.root = ET.fromstring(text)
        dd = _kid(self.root, "DataDictionary")
        self.valid = {}
        self.optype = {}
        for f in _kids(dd, "DataField"):
            self.optype[f.get("name")] = f.get("optype")
            vals = [v.get("value") for v in _kids(f, "Value")]
            if vals:
                self.valid[f.get("name")] = set(vals)
        self.model = next(c for c in self.root if _strip(c.tag) in
                          ("NeuralNetwork", "RegressionModel", "TreeModel", "MiningModel"))

    # ---- fields -------------------------------------------------------------------------
    def _schema_values(self, model, rec: dict) -> dict:
        """Raw record -> model field values after the MiningSchema (None = missing)."""
        out = {}
        ms = _kid(model, "MiningSchema")
        for mf in _kids(ms, "MiningField") if ms is not None else []:
            name = mf.get("name")
            if mf.get("usageType") == "target":
                continue
            v = rec.get(name)
            if isinstance(v, str) and v.strip() == "":
                v = None
            if v is not None and self.optype.get(name) == "continuous":
                v = _num(v)
            elif v is not None:
                v = str(v).strip()
                if name in self.valid and v not in self.valid[name] and mf.get("invalidValueTreatment") == "asMissing":
                    v = None
            if v is None and mf.get("missingValueReplacement") is not None:
                r = mf.get("missingValueReplacement")
                v = _num(r) if self.optype.get(name) == "continuous" else r
            out[name] = v
        return out

    def _derive(self, model, vals: dict) -> dict:
        lt = _kid(model, "LocalTransformations")
        for df in _kids(lt, "DerivedField") if lt is not None else []:
            vals[df.get("name")] = self._expr(list(df)[0], vals)
        return vals

    def _expr(self, e, vals):
        t = _strip(e.tag)
        if t == "FieldRef":
            return vals.get(e.get("field"))
        if t == "NormContinuous":
            x = vals.get(e.get("field"))
            if x is None:
                return _num(e.get("mapMissingTo"))
            pts = [(float(p.get("orig")), float(p.get("norm"))) for p in _kids(e, "LinearNorm")]
            if x <= pts[0][0]:
                return pts[0][1] if e.get("outliers") == "asExtremeValues" else \
                    pts[0][1] + (x - pts[0][0]) * (pts[1][1] - pts[0][1]) / (pts[1][0] - pts[0][0])
            if x >= pts[-1][0]:
                return pts[-1][1] if e.get("outliers") == "asExtremeValues" else \
                    pts[-1][1] + (x - pts[-1][0]) * (pts[-1][1] - pts[-2][1]) / (pts[-1][0] - pts[-2][0])
            for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
                if x0 <= x <= x1:
                    return y0 + (x - x0) * (y1 - y0) / (x1 - x0)
        if t == "MapValues":
            pair = _kid(e, "FieldColumnPair")
            x = vals.get(pair.get("field"))
            if x is None:
                return _num(e.get("mapMissingTo"))
            col, out = pair.get("column"), e.get("outputColumn")
            for row in _kids(_kid(e, "InlineTable"), "row"):
                cells = {_strip(c.tag): (c.text or "") for c in row}
                if cells.get(col) == str(x):
                    return _num(cells.get(out))
            return _num(e.get("defaultValue"))
        if t == "Discretize":
            x = vals.get(e.get("field"))
            if x is None:
                return _num(e.get("mapMissingTo"))
            for b in _kids(e, "DiscretizeBin"):
                iv = _kid(b, "Interval")
                lo, hi = _num(iv.get("leftMargin")), _num(iv.get("rightMargin"))
                cl = iv.get("closure", "closedOpen")
                ok_lo = lo is None or (x >= lo if cl.startswith("closed") else x > lo)
                ok_hi = hi is None or (x <= hi if cl.endswith("Closed") else x < hi)
                if ok_lo and ok_hi:
                    return _num(b.get("binValue"))
            return _num(e.get("defaultValue"))
        if t == "Constant":
            v = _num(e.text)
            return v if v is not None else (e.text or "").strip()
        if t == "Apply":
            args = [self._expr(c, vals) for c in e if _strip(c.tag) != "Extension"]
            fn = e.get("function")
            if any(a is None for a in args) and fn not in ("isMissing", "isNotMissing", "if"):
                return _num(e.get("mapMissingTo"))
            f2 = {"+": lambda a, b: a + b, "-": lambda a, b: a - b, "*": lambda a, b: a * b,
                  "/": lambda a, b: a / b if b != 0 else None, "pow": lambda a, b: a ** b,
                  "min": min, "max": max}
            if fn in f2:
                r = args[0]
                for a in args[1:]:
                    r = f2[fn](r, a)
                return r
            f1 = {"log10": math.log10, "ln": math.log, "exp": math.exp, "sqrt": math.sqrt, "abs": abs,
                  "floor": math.floor, "ceil": math.ceil, "round": round}
            if fn in f1:
                return float(f1[fn](args[0]))
            if fn == "isMissing":
                return args[0] is None
            if fn == "isNotMissing":
                return args[0] is not None
            if fn == "if":
                return args[1] if args[0] else (args[2] if len(args) > 2 else None)
            raise ValueError(f"unsupported PMML function {fn}")
        raise ValueError(f"unsupported PMML expression {t}")

    # ---- models -------------------------------------------------------------------------
    def _eval(self, model, rec: dict) -> float:
        vals = self._derive(model, self._schema_values(model, rec))
        t = _strip(model.tag)
        if t == "NeuralNetwork":
            act0 = model.get("activationFunction", "logistic")
            neurons = {}
            for ni in _kids(_kid(model, "NeuralInputs"), "NeuralInput"):
                df = _kid(ni, "DerivedField")
                neurons[ni.get("id")] = self._expr(list(df)[0], vals)
            last = []
            for layer in _kids(model, "NeuralLayer"):
                f = _ACT[layer.get("activationFunction", act0)]
                last = []
                for n in _kids(layer, "Neuron"):
                    z = float(n.get("bias", 0.0)) + sum(float(c.get("weight")) * neurons[c.get("from")]
                                                        for c in _kids(n, "Con"))
                    neurons[n.get("id")] = f(z)
                    last.append(n.get("id"))
            out = _kid(_kid(model, "NeuralOutputs"), "NeuralOutput")
            return neurons[out.get("outputNeuron")]
        if t == "RegressionModel":
            rt = _kid(model, "RegressionTable")
            z = float(rt.get("intercept", 0.0))
            for p in _kids(rt, "NumericPredictor"):
                z += float(p.get("coefficient")) * (vals[p.get("name")] ** int(p.get("exponent", 1)))
            nm = model.get("normalizationMethod", "none")
            return 1.0 / (1.0 + math.exp(-z)) if nm == "logit" else z
        if t == "TreeModel":
            node = _kid(model, "Node")
            while True:
                nxt = None
                for ch in _kids(node, "Node"):
                    if self._pred(list(ch)[0], vals):
                        nxt = ch
                        break
                if nxt is None:
                    return float(node.get("score"))
                node = nxt
        if t == "MiningModel":
            seg = _kid(model, "Segmentation")
            method = seg.get("multipleModelMethod")
            ys, ws = [], []
            for s in _kids(seg, "Segment"):
                if not self._pred(list(s)[0], vals):
                    continue
                sub = next(c for c in s if _strip(c.tag) in ("NeuralNetwork", "RegressionModel", "TreeModel",
                                                            "MiningModel"))
                ys.append(self._eval(sub, rec))
                ws.append(float(s.get("weight", 1.0)))
            ys, ws = np.asarray(ys), np.asarray(ws)
            if method == "sum":
                return float(ys.sum())
            if method == "weightedSum":
                return float((ys * ws).sum())
            if method == "average":
                return float(ys.mean())
            if method == "weightedAverage":
                return float((ys * ws).sum() / ws.sum())
            raise ValueError(f"unsupported multipleModelMethod {method}")
        raise ValueError(f"unsupported model {t}")

    def _pred(self, p, vals) -> bool:
        t = _strip(p.tag)
        if t == "True":
            return True
        if t == "False":
            return False
        if t == "SimplePredicate":
            x, op = vals.get(p.get("field")), p.get("operator")
            if op == "isMissing":
                return x is None
            if op == "isNotMissing":
                return x is not None
            if x is None:
                return False
            v = p.get("value")
            if isinstance(x, float):
                v = float(v)
            return {"lessThan": x < v, "lessOrEqual": x <= v, "greaterThan": x > v, "greaterOrEqual": x >= v,
                    "equal": x == v, "notEqual": x != v}[op]
        if t == "SimpleSetPredicate":
            x = vals.get(p.get("field"))
            if x is None:
                return False
            arr = _kid(p, "Array")
            items = set(shlex.split(arr.text or "")) if arr.text else set()
            inside = str(x) in items
            return inside if p.get("booleanOperator") == "isIn" else not inside
        if t == "CompoundPredicate":
            rs = [self._pred(c, vals) for c in p]
            op = p.get("booleanOperator")
            return any(rs) if op == "or" else all(rs) if op == "and" else (sum(rs) % 2 == 1)
        raise ValueError(f"unsupported predicate {t}")

    def evaluate(self, records) -> np.ndarray:
        """[N] predictions for a list of records ({field: raw value})."""
        return np.array([self._eval(self.model, r) for r in records], dtype=np.float64)

    def output_fields(self) -> list:
        out = _kid(self.model, "Output")
        return [f.get("name") for f in _kids(out, "OutputField")] if out is not None else []

    def evaluate_outputs(self, records) -> dict:
        """The model's ``Output`` fields per record: ``predictedValue`` (the raw prediction) and
        ``transformedValue`` (its expression, e.g. Shifu's RawResult x 1000 NormContinuous,
        PMMLTranslator's score scaling) -> {name: [N] array}.  Without an Output element:
        {"predicted": evaluate(records)}."""
        out = _kid(self.model, "Output")
        if out is None:
            return {"predicted": self.evaluate(records)}
        fields = _kids(out, "OutputField")
        res = {f.get("name"): np.empty(len(records)) for f in fields}
        for i, r in enumerate(records):
            y = self._eval(self.model, r)
            vals = {}
            for f in fields:
                feat = f.get("feature", "predictedValue")
                if feat == "predictedValue":
                    v = y
                elif feat == "transformedValue":
                    ex = [c for c in f if _strip(c.tag) != "Extension"]
                    v = self._expr(ex[0], vals) if ex else y
                else:
                    raise ValueError(f"unsupported OutputField feature {feat}")
                vals[f.get("name")] = v
                res[f.get("name")][i] = np.nan if v is None else float(v)
        return res


def records_from_table(table, names) -> list:
    """RawTable -> list of {name: raw value} (strings for categorical, float/None for numeric)."""
    cols = {}
    for n in names:
        c = table[n]
        if c.kind == "str":
            cols[n] = [None if s == "" else s for s in c.strings()]
        else:
            cols[n] = [None if v != v else float(v) for v in c.values]
    n = table.n
    return [{k: v[i] for k, v in cols.items()} for i in range(n)]
