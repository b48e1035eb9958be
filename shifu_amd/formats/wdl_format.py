"""``.wdl`` model files in the reference's binary layout (I4).

``BinaryWDLSerializer.save(modelConfig, columnConfigList, wnd, ...)``
(J/core/dtrain/wdl/BinaryWDLSerializer.java:57-108), read back by
``IndependentWDLModel.loadFromStream`` (J/core/dtrain/wdl/IndependentWDLModel.java:198-300);
gzip, Java ``DataOutput`` big-endian:

    int    WDL_FORMAT_VERSION (1)
    float 0, float 0, double 0, UTF "Reserved field"
    string normType                      (StringUtils.writeString: int length + UTF-8)
    int    #columns, NNColumnStats * n    (the selected / good-candidate input columns)
    WideAndDeep.write (WideAndDeep.java:558-612):
      int serializationType (0 WEIGHTS, 1 GRADIENTS, 2 MODEL_SPEC)
      bool+DenseInputLayer{int out}
      int #hidden, DenseLayer{float l2, int in, int out, bool+float[in][out] W, bool+float[out] b} * n
      bool+DenseLayer final (out = 1)
      bool+EmbedLayer{int n, EmbedFieldLayer{int colId, int in, int out, bool+float[in][out]} * n}
      bool+WideLayer{int n, WideFieldLayer{int colId, float l2, int in, bool+float[in]} * n,
                     bool+WideDenseLayer{float l2, int in, bool+float[in]}, bool+BiasLayer{float}}
      int #acts, UTF act * n
      MODEL_SPEC only: int n, (int colId, int cateSize) * n, int numericalSize,
                       intList denseColumnIds, embedColumnIds, embedOutputs, wideColumnIds,
                       hiddenNodes, float l2reg
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .javaio import JavaIn, JavaOut
from .nn_format import read_column_stats, write_column_stats

WDL_FORMAT_VERSION = 1
WEIGHTS, GRADIENTS, MODEL_SPEC = 0, 1, 2


@dataclass
class WDLSpec:
    """Parameters of one WideAndDeep network in the reference's orientation."""
    n_dense: int
    dense_ids: list
    embed_ids: list
    embed_outputs: list
    wide_ids: list
    cate_sizes: dict                      # column id -> number of slots of its wide/embed table
    hidden: list
    acts: list
    l2reg: float = 0.0
    hidden_W: list = field(default_factory=list)    # [in][out] each
    hidden_b: list = field(default_factory=list)
    final_W: np.ndarray | None = None               # [in][1]
    final_b: np.ndarray | None = None               # [1]
    embed_W: list = field(default_factory=list)     # [cate][dim] per embed id
    wide_W: list = field(default_factory=list)      # [cate] per wide id
    wide_dense: np.ndarray | None = None            # [n_dense]
    bias: float | None = None
    wide_on: bool = True
    deep_on: bool = True


def _f2(o: JavaOut, a):
    if a is None:
        o.bool(False)
        return
    a = np.asarray(a, dtype=">f4")
    o.bool(True)
    o.raw(a.tobytes())


def _r2(i: JavaIn, n: int):
    if not i.bool():
        return None
    return np.frombuffer(i._take(4 * n), dtype=">f4").astype(np.float32)


def _int_list(o: JavaOut, a):
    o.int(len(a))
    for v in a:
        o.int(int(v))


def _read_int_list(i: JavaIn):
    return [i.int() for _ in range(i.int())]


def write_wdl_file(path: str, norm_type: str, col_stats: list, spec: WDLSpec, ser_type: int = MODEL_SPEC):
    o = JavaOut()
    o.int(WDL_FORMAT_VERSION)
    o.float(0.0)
    o.float(0.0)
    o.double(0.0)
    o.utf("Reserved field")
    o.string(norm_type)
    o.int(len(col_stats))
    for cs in col_stats:
        write_column_stats(o, cs)
    # WideAndDeep.write
    o.int(ser_type)
    o.bool(True)
    o.int(spec.n_dense)                                       # DenseInputLayer
    if spec.deep_on:
        o.int(len(spec.hidden_W))
        for W, b in zip(spec.hidden_W, spec.hidden_b):
            o.float(spec.l2reg)
            o.int(W.shape[0])
            o.int(W.shape[1])
            _f2(o, W)
            _f2(o, b)
        o.bool(True)
        o.float(spec.l2reg)
        o.int(spec.final_W.shape[0])
        o.int(1)
        _f2(o, spec.final_W)
        _f2(o, spec.final_b)
        o.bool(True)                                          # EmbedLayer
        o.int(len(spec.embed_W))
        for cid, W in zip(spec.embed_ids, spec.embed_W):
            o.int(cid)
            o.int(W.shape[0])
            o.int(W.shape[1])
            _f2(o, W)
    else:
        o.int(0)
        o.bool(False)
        o.bool(False)
    if spec.wide_on:
        o.bool(True)                                          # WideLayer
        o.int(len(spec.wide_W))
        for cid, w in zip(spec.wide_ids, spec.wide_W):
            o.int(cid)
            o.float(spec.l2reg)
            o.int(len(w))
            _f2(o, w)
        o.bool(True)
        o.float(spec.l2reg)
        o.int(spec.n_dense)
        _f2(o, spec.wide_dense)
        o.bool(True)
        o.float(0.0 if spec.bias is None else spec.bias)
    else:
        o.bool(False)
    acts = spec.acts if spec.deep_on else []
    o.int(len(acts))
    for a in acts:
        o.utf(a)
    if ser_type == MODEL_SPEC:
        o.int(len(spec.cate_sizes))
        for k, v in spec.cate_sizes.items():
            o.int(int(k))
            o.int(int(v))
        o.int(spec.n_dense)
        for lst in (spec.dense_ids, spec.embed_ids, spec.embed_outputs, spec.wide_ids, spec.hidden):
            _int_list(o, lst)
        o.float(spec.l2reg)
    with open(path, "wb") as f:
        f.write(o.gzip_bytes())


def read_wdl_file(path: str):
    """-> (version, norm_type, [NNColumnStats], WDLSpec)."""
    with open(path, "rb") as f:
        i = JavaIn(f.read())
    version = i.int()
    i.float()
    i.float()
    i.double()
    i.utf()
    norm = i.string()
    stats = [read_column_stats(i) for _ in range(i.int())]
    ser = i.int()
    n_dense = i.int() if i.bool() else 0
    hidden_W, hidden_b = [], []
    l2 = 0.0
    for _ in range(i.int()):
        l2 = i.float()
        a, b = i.int(), i.int()
        W = _r2(i, a * b)
        hidden_W.append(None if W is None else W.reshape(a, b))
        hidden_b.append(_r2(i, b))
    final_W = final_b = None
    if i.bool():
        l2 = i.float()
        a, b = i.int(), i.int()
        W = _r2(i, a * b)
        final_W = None if W is None else W.reshape(a, b)
        final_b = _r2(i, b)
    embed_ids, embed_W = [], []
    if i.bool():
        for _ in range(i.int()):
            cid, a, b = i.int(), i.int(), i.int()
            W = _r2(i, a * b)
            embed_ids.append(cid)
            embed_W.append(None if W is None else W.reshape(a, b))
    wide_ids, wide_W, wide_dense, bias, wide_on = [], [], None, None, False
    if i.bool():
        wide_on = True
        for _ in range(i.int()):
            cid = i.int()
            i.float()
            n = i.int()
            wide_ids.append(cid)
            wide_W.append(_r2(i, n))
        if i.bool():
            i.float()
            wide_dense = _r2(i, i.int())
        if i.bool():
            bias = i.float()
    acts = [i.utf() for _ in range(i.int())]
    cate_sizes, dense_ids, embed_outputs, hidden = {}, [], [], []
    if ser == MODEL_SPEC:
        for _ in range(i.int()):
            k = i.int()
            cate_sizes[k] = i.int()
        n_dense = i.int()
        dense_ids = _read_int_list(i)
        embed_ids = _read_int_list(i) or embed_ids
        embed_outputs = _read_int_list(i)
        wide_ids = _read_int_list(i) or wide_ids
        hidden = _read_int_list(i)
        l2 = i.float()
    spec = WDLSpec(n_dense, dense_ids, embed_ids, embed_outputs, wide_ids, cate_sizes,
                   hidden or [W.shape[1] for W in hidden_W if W is not None], acts, l2, hidden_W, hidden_b,
                   final_W, final_b, embed_W, wide_W, wide_dense, bias, wide_on, final_W is not None)
    return version, norm, stats, spec
