"""``.nn`` model files (I1).

* Encog EG text (``encog,BasicNetwork,java,3.0.0,...``), written by
  ``NNOutput.writeEncogModelToFileSystem`` (J/core/dtrain/nn/NNOutput.java:402-416); fixture
  ``src/test/resources/example/cancer-judgement/ModelStore/ModelSet1/models/model0.nn``.
* Binary v1 (gzip): ``BinaryNNSerializer.save`` (J/core/dtrain/nn/BinaryNNSerializer.java:46-108),
  ``NNColumnStats.write`` and ``PersistBasicFloatNetwork.saveNetwork``
  (J/core/dtrain/dataset/PersistBasicFloatNetwork.java:280-350); layout in SURVEY Appendix B.

Encog flat layout: layers output-first; layerCounts include the bias neuron of every
non-output layer; weight block l (to = layer l, from = layer l+1) is row-major [to][from+1].
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from .javaio import JavaIn, JavaOut

ACT_CLASS = {"sigmoid": "ActivationSigmoid", "tanh": "ActivationTANH", "linear": "ActivationLinear",
             "relu": "ActivationReLU", "leakyrelu": "ActivationLeakyReLU", "swish": "ActivationSwish",
             "ptanh": "ActivationPTANH", "log": "ActivationLOG", "sin": "ActivationSIN"}
CLASS_ACT = {v.lower(): k for k, v in ACT_CLASS.items()}
ACT_PARAMS = {"relu": [0.0, 0.0], "leakyrelu": [0.0, 0.01]}
SUBSET_PROP = "shifu.nn.feature.subset"     # input positions a feature-subsampled bag was trained on


def act_from_class(name: str) -> str:
    n = name.strip().strip('"').split("|")[0].split(".")[-1].lower()
    return CLASS_ACT.get(n, "sigmoid")


@dataclass
class NNNetwork:
    """Input-first description: sizes [n_in, h1, ..., n_out], acts per non-input layer,
    weights[l] = [out_l, in_l + 1] (bias last)."""
    sizes: list
    acts: list
    weights: list
    properties: dict = field(default_factory=dict)
    feature_set: list = field(default_factory=list)

    @property
    def n_in(self):
        return self.sizes[0]

    @property
    def n_out(self):
        return self.sizes[-1]

    def input_subset(self):
        """Input positions of a feature-subsampled network (None = all inputs)."""
        if self.feature_set and len(self.feature_set) == self.n_in:
            return list(self.feature_set)
        v = (self.properties or {}).get(SUBSET_PROP)
        return [int(t) for t in str(v).split(",") if t.strip()] if v else None

    # ---- Encog flat ---------------------------------------------------------------------
    def flat(self):
        L = len(self.sizes)
        sizes_of = list(reversed(self.sizes))              # output-first
        feed = sizes_of[:]
        counts = [feed[0]] + [c + 1 for c in feed[1:]]      # bias on every non-output layer
        layer_index, acc = [], 0
        for c in counts:
            layer_index.append(acc)
            acc += c
        layer_output = [0.0] * acc
        for i in range(1, L):
            layer_output[layer_index[i] + feed[i]] = 1.0
        weight_index, w, acc = [], [], 0
        for i in range(L - 1):
            weight_index.append(acc)
            blk = np.asarray(self.weights[L - 2 - i], dtype=np.float64)   # to=layer(L-1-i) input-first
            w.append(blk.reshape(-1))
            acc += blk.size
        weight_index.append(acc)
        acts_of = list(reversed(self.acts)) + ["linear"]   # input layer activation = linear
        return dict(beginTraining=0, connectionLimit=0.0, contextTargetOffset=[0] * L, contextTargetSize=[0] * L,
                    endTraining=L - 1, hasContext=False, inputCount=self.n_in, layerCounts=counts,
                    layerFeedCounts=feed, layerContextCount=[0] * L, layerIndex=layer_index,
                    output=layer_output, outputCount=self.n_out, weightIndex=weight_index,
                    weights=np.concatenate(w) if w else np.zeros(0),
                    biasActivation=[0.0] + [1.0] * (L - 1), acts=acts_of)

    @staticmethod
    def from_flat(layer_feed_counts, weights, acts_output_first, weight_index=None, props=None, features=None):
        feed = list(layer_feed_counts)
        L = len(feed)
        sizes = list(reversed(feed))
        ws = []
        pos = 0
        blocks = []
        for i in range(L - 1):
            to, frm = feed[i], feed[i + 1]
            n = to * (frm + 1)
            start = weight_index[i] if weight_index else pos
            blocks.append(np.asarray(weights[start: start + n], dtype=np.float64).reshape(to, frm + 1))
            pos = start + n
        ws = list(reversed(blocks))
        acts = [act_from_class(a) for a in reversed(acts_output_first[:L - 1])]
        return NNNetwork(sizes, acts, ws, props or {}, features or [])

    # ---- forward (double precision oracle = IndependentNNModel semantics) -------------------
    def forward(self, x: np.ndarray) -> np.ndarray:
        from ..models.nn import act_fwd
        import torch
        a = np.asarray(x, dtype=np.float64)
        for l, W in enumerate(self.weights):
            z = a @ W[:, :-1].T + W[:, -1]
            a = act_fwd(self.acts[l], torch.from_numpy(z)).numpy()
        return a


# ---- Encog EG text -----------------------------------------------------------------------------
def _fmt(v):
    if isinstance(v, bool):
        return "t" if v else "f"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    f = float(v)
    return str(int(f)) if f == int(f) and abs(f) < 1e15 else repr(f)


def write_encog(net: NNNetwork, path: str):
    fl = net.flat()
    lines = [f"encog,BasicNetwork,java,3.0.0,1,{int(time.time() * 1000)}", "[BASIC]", "[BASIC:PARAMS]"]
    for k, v in (net.properties or {}).items():
        lines.append(f"{k}={v}")
    lines.append("[BASIC:NETWORK]")
    order = ["beginTraining", "connectionLimit", "contextTargetOffset", "contextTargetSize", "endTraining",
             "hasContext", "inputCount", "layerCounts", "layerFeedCounts", "layerContextCount", "layerIndex",
             "output", "outputCount", "weightIndex", "weights", "biasActivation"]
    for k in order:
        v = fl[k]
        if isinstance(v, (list, tuple, np.ndarray)):
            lines.append(f"{k}=" + ",".join(_fmt(x) for x in v))
        else:
            lines.append(f"{k}={_fmt(v)}")
    lines.append("[BASIC:ACTIVATION]")
    for a in fl["acts"]:
        lines.append(f'"{ACT_CLASS.get(a, "ActivationSigmoid")}"')
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def read_encog(path_or_text: str) -> NNNetwork:
    text = path_or_text
    if "\n" not in path_or_text:
        with open(path_or_text, encoding="utf-8") as f:
            text = f.read()
    section = None
    kv, acts, props = {}, [], {}
    for line in text.splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith("["):
            section = line
            continue
        if section == "[BASIC:NETWORK]" and "=" in line:
            k, v = line.split("=", 1)
            kv[k] = v
        elif section == "[BASIC:PARAMS]" and "=" in line:
            k, v = line.split("=", 1)
            props[k] = v
        elif section == "[BASIC:ACTIVATION]":
            acts.append(line.strip('"').split('"')[0])

    def ints(k):
        return [int(x) for x in kv[k].split(",")] if kv.get(k) else []

    def dbls(k):
        return np.array([float(x) for x in kv[k].split(",")]) if kv.get(k) else np.zeros(0)
    return NNNetwork.from_flat(ints("layerFeedCounts"), dbls("weights"), acts, ints("weightIndex"), props)


# ---- binary v1 ---------------------------------------------------------------------------------
@dataclass
class NNColumnStats:
    column_num: int
    column_name: str
    column_type: str               # A/N/C/H
    cutoff: float
    mean: float
    stddev: float
    woe_mean: float
    woe_stddev: float
    woe_wgt_mean: float
    woe_wgt_stddev: float
    bin_boundaries: list
    bin_categories: list
    bin_pos_rates: list
    bin_count_woes: list
    bin_weight_woes: list


TYPE_BYTE = {"A": 0, "N": 1, "C": 2, "H": 3}
BYTE_TYPE = {v: k for k, v in TYPE_BYTE.items()}


def _save_network(o: JavaOut, net: NNNetwork):
    fl = net.flat()
    o.int(len(net.properties or {}))
    for k, v in (net.properties or {}).items():
        o.string(str(k))
        o.string(str(v))
    o.int(fl["beginTraining"])
    o.double(fl["connectionLimit"])
    o.int_array(fl["contextTargetOffset"])
    o.int_array(fl["contextTargetSize"])
    o.int(fl["endTraining"])
    o.bool(fl["hasContext"])
    o.int(fl["inputCount"])
    o.int_array(fl["layerCounts"])
    o.int_array(fl["layerFeedCounts"])
    o.int_array(fl["layerContextCount"])
    o.int_array(fl["layerIndex"])
    o.double_array(fl["output"])
    o.int(fl["outputCount"])
    o.int_array(fl["weightIndex"])
    o.double_array(fl["weights"])
    o.double_array(fl["biasActivation"])
    o.int(len(fl["acts"]))
    for a in fl["acts"]:
        o.string(ACT_CLASS.get(a, "ActivationSigmoid"))
        o.double_array(ACT_PARAMS.get(a, []))
    fs = net.feature_set or []
    o.int(len(fs))
    for f in fs:
        o.int(f)


def _load_network(i: JavaIn) -> NNNetwork:
    props = {}
    for _ in range(i.int()):
        k = i.string()
        props[k] = i.string()
    i.int(); i.double(); i.int_array(); i.int_array(); i.int(); i.bool(); i.int()
    i.int_array()                           # layerCounts
    feed = i.int_array()
    i.int_array(); i.int_array()            # context count, layer index
    i.double_array()                        # layer output
    i.int()                                 # output count
    widx = i.int_array()
    w = i.double_array()
    i.double_array()                        # bias activation
    acts = []
    for _ in range(i.int()):
        acts.append(i.string())
        i.double_array()
    feats = [i.int() for _ in range(i.int())]
    return NNNetwork.from_flat(feed, w, acts, widx, props, feats)


def write_column_stats(o: JavaOut, cs: NNColumnStats):
    """NNColumnStats.write (J/core/dtrain/nn/NNColumnStats.java:97-124)."""
    o.int(cs.column_num)
    o.string(cs.column_name)
    o.byte(TYPE_BYTE.get(cs.column_type or "N", 1))
    for v in (cs.cutoff, cs.mean, cs.stddev, cs.woe_mean, cs.woe_stddev, cs.woe_wgt_mean, cs.woe_wgt_stddev):
        o.double(0.0 if v is None else v)
    o.double_array(cs.bin_boundaries)
    cats = cs.bin_categories or []
    o.int(len(cats))
    for c in cats:
        o.string(c)
    o.double_array(cs.bin_pos_rates)
    o.double_array(cs.bin_count_woes)
    o.double_array(cs.bin_weight_woes)


def read_column_stats(i: JavaIn) -> NNColumnStats:
    num = i.int()
    name = i.string()
    typ = BYTE_TYPE.get(i.byte(), "N")
    vals = [i.double() for _ in range(7)]
    bb = i.double_array()
    cats = [i.string() for _ in range(i.int())]
    pr, cw, ww = i.double_array(), i.double_array(), i.double_array()
    return NNColumnStats(num, name, typ, *vals, bb, cats, pr, cw, ww)


def write_binary_nn(path: str, norm_type: str, col_stats: list, column_mapping: dict, networks: list):
    o = JavaOut()
    o.int(1)
    o.string(norm_type)
    o.int(len(col_stats))
    for cs in col_stats:
        write_column_stats(o, cs)
    o.int(len(column_mapping))
    for k, v in column_mapping.items():
        o.int(k)
        o.int(v)
    o.int(len(networks))
    for net in networks:
        _save_network(o, net)
    with open(path, "wb") as f:
        f.write(o.gzip_bytes())


def read_binary_nn(path: str):
    with open(path, "rb") as f:
        i = JavaIn(f.read())
    version = i.int()
    norm = i.string()
    stats = [read_column_stats(i) for _ in range(i.int())]
    mapping = {}
    for _ in range(i.int()):
        k = i.int()
        mapping[k] = i.int()
    nets = [_load_network(i) for _ in range(i.int())]
    return {"version": version, "norm_type": norm, "column_stats": stats, "column_mapping": mapping,
            "networks": nets}


def is_binary_nn(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(2) == b"\x1f\x8b"
