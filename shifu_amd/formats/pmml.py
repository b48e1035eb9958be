"""PMML 4.2 export (I7) for NN, LR and tree ensembles with local transformations.

``PMMLTranslator.build`` (J/core/pmml/PMMLTranslator.java:77) + the creators under
``J/core/pmml/builder/impl`` (DataDictionary, MiningSchema, local z-score / WOE transforms,
NeuralNetwork / Regression / MiningModel(TreeModel) bodies).  Normalization is expressed as
``DerivedField``s so a PMML engine reproduces ``Normalizer`` on raw inputs:
* ZSCALE numeric: clip to mean +- cutoff*std then ``NormContinuous`` linear map ((x-mean)/std);
  missing -> mean (``mapMissingTo``).
* categorical: ``MapValues`` from category to pos-rate z-score or WOE (missing -> last bin).
* WOE numeric: ``Discretize`` bins -> WOE.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

import numpy as np

from ..algos.normalize import STD_DEV_CUTOFF, woe_mean_std, zscore

ACT_PMML = {"sigmoid": "logistic", "tanh": "tanh", "linear": "identity", "relu": "rectifier",
            "leakyrelu": "rectifier", "log": "identity", "sin": "sine", "ptanh": "tanh", "swish": "identity"}


def _root():
    pmml = ET.Element("PMML", version="4.2", xmlns="http://www.dmg.org/PMML-4_2")
    ET.SubElement(pmml, "Header", copyright="shifu_amd", description="exported by shifu_amd")
    return pmml


def _data_dictionary(pmml, cols, target):
    dd = ET.SubElement(pmml, "DataDictionary", numberOfFields=str(len(cols) + 1))
    for c in cols:
        if c.is_categorical():
            f = ET.SubElement(dd, "DataField", name=c.name, optype="categorical", dataType="string")
            for v in c.bin_category or []:
                for s in str(v).split("^"):
                    ET.SubElement(f, "Value", value=s)
        else:
            ET.SubElement(dd, "DataField", name=c.name, optype="continuous", dataType="double")
    ET.SubElement(dd, "DataField", name=target, optype="continuous", dataType="double")


def _mining_schema(model, cols, target):
    ms = ET.SubElement(model, "MiningSchema")
    for c in cols:
        ET.SubElement(ms, "MiningField", name=c.name, optype="categorical" if c.is_categorical() else "continuous",
                      usageType="active")
    ET.SubElement(ms, "MiningField", name=target, usageType="target")


def _transforms(model, cols, norm_type: str, cutoff: float):
    """-> list of derived field names (model inputs in column order)."""
    lt = ET.SubElement(model, "LocalTransformations")
    names = []
    nt = (norm_type or "ZSCALE").upper()
    for c in cols:
        dn = f"{c.name}_norm"
        df = ET.SubElement(lt, "DerivedField", name=dn, optype="continuous", dataType="double")
        if c.is_categorical():
            mv = ET.SubElement(df, "MapValues", outputColumn="out", dataType="double")
            if "WOE" in nt:
                vals = np.asarray(c.bin_count_woe if "WEIGHT" not in nt else c.bin_weighted_woe, dtype=float)
                if "ZSCALE" in nt or "ZSCORE" in nt:
                    m, s = woe_mean_std(c, "WEIGHT" in nt)
                    vals = zscore(vals, m, s, cutoff)
            else:
                vals = zscore(np.asarray(c.bin_pos_rate, dtype=float), c.mean, c.std_dev, cutoff)
            mv.set("mapMissingTo", repr(float(vals[-1])))
            mv.set("defaultValue", repr(float(vals[-1])))
            ET.SubElement(mv, "FieldColumnPair", field=c.name, column="origin")
            it = ET.SubElement(mv, "InlineTable")
            for i, v in enumerate(c.bin_category or []):
                for s in str(v).split("^"):
                    row = ET.SubElement(it, "row")
                    ET.SubElement(row, "origin").text = s
                    ET.SubElement(row, "out").text = repr(float(vals[i]))
        elif "WOE" in nt:
            vals = np.asarray(c.bin_count_woe if "WEIGHT" not in nt else c.bin_weighted_woe, dtype=float)
            if "ZSCALE" in nt or "ZSCORE" in nt:
                m, s = woe_mean_std(c, "WEIGHT" in nt)
                vals = zscore(vals, m, s, cutoff)
            dz = ET.SubElement(df, "Discretize", field=c.name, mapMissingTo=repr(float(vals[-1])),
                               defaultValue=repr(float(vals[-1])))
            bb = list(c.bin_boundary or [])
            for i, lo in enumerate(bb):
                hi = bb[i + 1] if i + 1 < len(bb) else None
                b = ET.SubElement(dz, "DiscretizeBin", binValue=repr(float(vals[i])))
                iv = ET.SubElement(b, "Interval", closure="closedOpen")
                if lo != float("-inf"):
                    iv.set("leftMargin", repr(float(lo)))
                if hi is not None:
                    iv.set("rightMargin", repr(float(hi)))
        else:
            mean, std = float(c.mean or 0.0), float(c.std_dev or 0.0)
            nc = ET.SubElement(df, "NormContinuous", field=c.name, mapMissingTo="0.0", outliers="asExtremeValues")
            lo, hi = mean - cutoff * std, mean + cutoff * std
            if std > 1e-5:
                ET.SubElement(nc, "LinearNorm", orig=repr(lo), norm=repr((lo - mean) / std))
                ET.SubElement(nc, "LinearNorm", orig=repr(hi), norm=repr((hi - mean) / std))
            else:
                ET.SubElement(nc, "LinearNorm", orig=repr(mean - 1.0), norm="0.0")
                ET.SubElement(nc, "LinearNorm", orig=repr(mean + 1.0), norm="0.0")
        names.append(dn)
    return names


def _output(model, name="FinalResult"):
    out = ET.SubElement(model, "Output")
    ET.SubElement(out, "OutputField", name=name, feature="predictedValue")


# activations PMML 4.2 can express exactly; the others (log, swish, leaky ReLU, ptanh) have no
# PMML activationFunction, so such networks are refused instead of exported with wrong scores
PMML_EXACT_ACTS = {"sigmoid", "tanh", "linear", "relu", "sin"}


def _nn_element(parent, net, cols, target, norm_type, cutoff, model_name):
    """NeuralNetwork element (MiningSchema, Output, LocalTransformations, layers) under ``parent``."""
    bad = [a for a in net.acts if str(a).lower() not in PMML_EXACT_ACTS]
    if bad:
        raise ValueError(f"activation(s) {sorted(set(bad))} have no exact PMML 4.2 activationFunction")
    nn = ET.SubElement(parent, "NeuralNetwork", modelName=model_name, functionName="regression",
                       activationFunction="logistic", numberOfLayers=str(len(net.weights)))
    _mining_schema(nn, cols, target)
    _output(nn)
    inputs = _transforms(nn, cols, norm_type, cutoff)
    sub = net.input_subset()
    if sub is not None and len(inputs) != net.n_in:
        inputs = [inputs[i] for i in sub]
    ni = ET.SubElement(nn, "NeuralInputs", numberOfInputs=str(len(inputs)))
    prev = []
    for i, dn in enumerate(inputs):
        e = ET.SubElement(ni, "NeuralInput", id=f"0,{i}")
        df = ET.SubElement(e, "DerivedField", optype="continuous", dataType="double")
        ET.SubElement(df, "FieldRef", field=dn)
        prev.append(f"0,{i}")
    for l, W in enumerate(net.weights):
        W = np.asarray(W)
        layer = ET.SubElement(nn, "NeuralLayer", numberOfNeurons=str(W.shape[0]),
                              activationFunction=ACT_PMML.get(net.acts[l], "logistic"))
        cur = []
        for j in range(W.shape[0]):
            nid = f"{l + 1},{j}"
            ne = ET.SubElement(layer, "Neuron", id=nid, bias=repr(float(W[j, -1])))
            for k, src in enumerate(prev):
                ET.SubElement(ne, "Con", **{"from": src, "weight": repr(float(W[j, k]))})
            cur.append(nid)
        prev = cur
    no = ET.SubElement(nn, "NeuralOutputs", numberOfOutputs=str(len(prev)))
    for nid in prev:
        o = ET.SubElement(no, "NeuralOutput", outputNeuron=nid)
        df = ET.SubElement(o, "DerivedField", optype="continuous", dataType="double")
        ET.SubElement(df, "FieldRef", field=target)
    return nn


def nn_pmml(net, cols, target, norm_type="ZSCALE", cutoff=STD_DEV_CUTOFF, model_name="model0"):
    """One NN (input-first ``NNNetwork``) -> PMML NeuralNetwork."""
    pmml = _root()
    _data_dictionary(pmml, cols, target)
    _nn_element(pmml, net, cols, target, norm_type, cutoff, model_name)
    return pmml


def nn_bagging_pmml(nets, cols, target, norm_type="ZSCALE", cutoff=STD_DEV_CUTOFF, model_name="model"):
    """All bagging NNs as ONE PMML (``export -t baggingpmml``, PMMLTranslator.build with
    isOutBaggingToOne, J/core/pmml/PMMLTranslator.java:122-159): a regression MiningModel whose
    Segmentation averages one NeuralNetwork segment per bag (ids ``Segement<i>`` as the reference
    names them), each with its own MiningSchema and LocalTransformations."""
    pmml = _root()
    _data_dictionary(pmml, cols, target)
    mm = ET.SubElement(pmml, "MiningModel", modelName=model_name, functionName="regression")
    _mining_schema(mm, cols, target)
    _output(mm)
    seg = ET.SubElement(mm, "Segmentation", multipleModelMethod="average")
    for i, net in enumerate(nets):
        s = ET.SubElement(seg, "Segment", id=f"Segement{i}")
        ET.SubElement(s, "True")
        _nn_element(s, net, cols, target, norm_type, cutoff, f"{model_name}{i}")
    return pmml


def lr_pmml(weights, cols, target, norm_type="ZSCALE", cutoff=STD_DEV_CUTOFF, model_name="model0"):
    pmml = _root()
    _data_dictionary(pmml, cols, target)
    rm = ET.SubElement(pmml, "RegressionModel", modelName=model_name, functionName="regression",
                       normalizationMethod="logit")
    _mining_schema(rm, cols, target)
    _output(rm)
    inputs = _transforms(rm, cols, norm_type, cutoff)
    rt = ET.SubElement(rm, "RegressionTable", intercept=repr(float(weights[-1])))
    for dn, w in zip(inputs, weights[:-1]):
        ET.SubElement(rt, "NumericPredictor", name=dn, exponent="1", coefficient=repr(float(w)))
    return pmml


def _left_predicate(s, model):
    """Predicate of the left child of a split, matching ``TreeModelFile.predict_node``: numeric
    ``x < threshold`` (missing -> the column mean via the MiningField replacement); categorical
    ``x in L`` where L = the stored set (isLeft) or its complement, OR ``isMissing`` when the
    missing/unseen bin (index = #categories) is in L (unseen values are declared invalid ->
    asMissing in the MiningSchema)."""
    name = model.names[s.column]
    if s.ftype == 1:
        return ET.Element("SimplePredicate", field=name, operator="lessThan", value=repr(float(s.threshold)))
    cats = model.categories.get(s.column, [])
    ncat = len(cats)
    stored = set(s.categories or set())
    left = stored if s.is_left else set(range(ncat + 1)) - stored
    vals = [v for i in sorted(left) if i < ncat for v in str(cats[i]).split("^")]
    inset = ET.Element("SimpleSetPredicate", field=name, booleanOperator="isIn")
    arr = ET.SubElement(inset, "Array", n=str(len(vals)), type="string")
    arr.text = " ".join('"' + v.replace('"', '\\"') + '"' for v in vals)
    if ncat not in left:
        return inset
    comp = ET.Element("CompoundPredicate", booleanOperator="or")
    comp.append(inset)
    ET.SubElement(comp, "SimplePredicate", field=name, operator="isMissing")
    return comp


def _tree_nodes(parent, nd, model, pred):
    el = ET.SubElement(parent, "Node", id=str(nd.id), score=repr(float(nd.predict or 0.0)))
    el.append(pred if pred is not None else ET.Element("True"))
    if nd.is_leaf():
        return
    _tree_nodes(el, nd.left, model, _left_predicate(nd.split, model))
    _tree_nodes(el, nd.right, model, ET.Element("True"))      # first true child wins


def _tree_mining_schema(model_el, cols, target, model):
    """Missing numeric -> the stored column mean (IndependentTreeModel's numerical mean
    replacement); values outside a categorical DataField's Value list are treated as missing."""
    ms = ET.SubElement(model_el, "MiningSchema")
    for c in cols:
        f = ET.SubElement(ms, "MiningField", name=c.name, usageType="active",
                          optype="categorical" if c.is_categorical() else "continuous")
        if c.is_categorical():
            f.set("invalidValueTreatment", "asMissing")
        else:
            f.set("missingValueReplacement", repr(float(model.numerical_means.get(c.num, c.mean or 0.0) or 0.0)))
            f.set("invalidValueTreatment", "asMissing")
    ET.SubElement(ms, "MiningField", name=target, usageType="target")


def tree_pmml(model, cols, target, model_name="model0"):
    """TreeModelFile -> MiningModel with one TreeModel segment per tree (GBT: weighted sum with
    the learning rates; RF: weighted average)."""
    pmml = _root()
    _data_dictionary(pmml, cols, target)
    mm = ET.SubElement(pmml, "MiningModel", modelName=model_name, functionName="regression")
    _mining_schema(mm, cols, target)
    _output(mm)
    is_gbt = model.algorithm.upper() == "GBT"
    seg = ET.SubElement(mm, "Segmentation", multipleModelMethod="weightedSum" if is_gbt else "weightedAverage")
    k = 0
    for bag in model.bags:
        for t in bag:
            s = ET.SubElement(seg, "Segment", id=str(k), weight=repr(float(t.learning_rate)))
            ET.SubElement(s, "True")
            tm = ET.SubElement(s, "TreeModel", functionName="regression", splitCharacteristic="binarySplit")
            _tree_mining_schema(tm, cols, target, model)
            _tree_nodes(tm, t.root, model, None)
            k += 1
    return pmml


def write_pmml(pmml, path: str):
    ET.indent(pmml) if hasattr(ET, "indent") else None
    ET.ElementTree(pmml).write(path, encoding="utf-8", xml_declaration=True)
