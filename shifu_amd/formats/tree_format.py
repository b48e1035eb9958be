"""``.gbt`` / ``.rf`` binary tree models (I2), format version 4 (gzip).

Writer/reader of ``BinaryDTSerializer.save`` (J/core/dtrain/dt/BinaryDTSerializer.java:47-146),
``IndependentTreeModel.loadFromStream`` (J/core/dtrain/dt/IndependentTreeModel.java:818-1080) and
the records ``TreeNode.write`` (:204-234), ``Node.write`` (J/core/dtrain/dt/Node.java:583-626),
``Split.write`` (Split.java:153-176, CONTINUOUS=1 / CATEGORICAL=2), ``Predict.write`` and
``SimpleBitSet.write`` (int byte-length + bytes, bit = value % 8 of byte value >> 3).
Layout: SURVEY Appendix C.  Versions <= 3 (ungzipped, ``version < 4`` -> one bag, float wgtCnt
for <= 2) are read with the same code path.

Pre-versioned legacy layout (``read_legacy_tree_model``): the reference fixture
``TR/example/wdbc/wdbcModelSetLocal/models/model0.gbt`` predates the version field; its strings
are int-length framed (``StringUtils.writeString``), nodes carry impurity / a leaf flag / the
weight-count ratio, splits carry the column name and the feature-type enum name.  The reference's
own ``IndependentTreeModel.loadFromStream`` cannot read it (it expects ``readInt`` version +
``readUTF``); the layout was recovered from the bytes (header, 13 nodes, root weight, 13 feature
ids: exactly 1025 bytes) and is documented field by field on the reader.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .javaio import JavaIn, JavaOut

CONTINUOUS, CATEGORICAL = 1, 2
UTF_BYTES_MARKER = -1
MAX_CATEGORICAL_VAL_LEN = 10 * 1024
TREE_FORMAT_VERSION = 4


@dataclass
class Split:
    column: int
    ftype: int
    threshold: float = 0.0
    is_left: bool = True
    categories: set | None = None      # category indices in the stored (left or right) set


@dataclass
class Node:
    id: int
    gain: float = 0.0
    wgt_cnt: float = 0.0
    split: Split | None = None
    predict: float | None = None
    class_value: int = 0
    left: "Node | None" = None
    right: "Node | None" = None

    def is_leaf(self):
        return self.split is None or (self.left is None and self.right is None)


@dataclass
class TreeRecord:
    tree_id: int
    node_num: int
    root: Node
    learning_rate: float
    root_wgt_cnt: float = 0.0
    features: list = field(default_factory=list)


@dataclass
class TreeModelFile:
    algorithm: str                      # "GBT" | "RF"
    loss: str
    is_classification: bool
    is_one_vs_all: bool
    input_count: int
    numerical_means: dict               # columnNum -> mean
    names: dict                         # columnNum -> name
    categories: dict                    # columnNum -> list[str]
    column_mapping: dict                # columnNum -> input index
    bags: list                          # list[list[TreeRecord]]
    version: int = TREE_FORMAT_VERSION

    # ---- scoring (IndependentTreeModel.computeRegressionScore semantics) ---------------------
    def _cat_index(self, col, value):
        cats = self.categories.get(col)
        if cats is None:
            return -1
        m = self.__dict__.setdefault("_catmap", {}).get(col)
        if m is None:
            m = {}
            for j, c in enumerate(cats):
                for s in str(c).split("^"):
                    m.setdefault(s, j)
            self._catmap[col] = m
        return m.get(value, len(cats))

    def vectorize(self, rows: dict) -> dict:
        """{column name -> array of raw values} -> {columnNum -> float array} (missing numeric ->
        mean, categorical -> category index)."""
        out = {}
        for col, name in self.names.items():
            raw = rows.get(name)
            if raw is None:
                raise KeyError(f"missing input column {name}")
            if col in self.categories:
                out[col] = np.array([self._cat_index(col, "" if v is None else str(v).strip()) for v in raw],
                                    dtype=np.float64)
            else:
                vals = np.empty(len(raw))
                mean = self.numerical_means.get(col, 0.0)
                for i, v in enumerate(raw):
                    try:
                        f = float(v)
                        vals[i] = mean if f != f else f
                    except (TypeError, ValueError):
                        vals[i] = mean
                out[col] = vals
        return out

    def predict_node(self, node: Node, x: dict, i: int) -> Node:
        while node.split is not None and not (node.left is None and node.right is None):
            s = node.split
            v = x[s.column][i]
            if s.ftype == CONTINUOUS:
                node = node.left if v < s.threshold else node.right
            else:
                nc = len(self.categories.get(s.column, []))
                idx = nc if (v < 0 or v >= nc) else int(v + 0.1)
                inset = idx in (s.categories or set())
                node = (node.left if inset else node.right) if s.is_left else (node.right if inset else node.left)
        return node

    def score(self, x: dict, n: int, convert: str = "RAW") -> np.ndarray:
        out = np.zeros(n)
        is_gbt = self.algorithm.upper() == "GBT"
        for bag in self.bags:
            p = np.zeros(n)
            wsum = 0.0
            for t in bag:
                for i in range(n):
                    nd = self.predict_node(t.root, x, i)
                    val = float(nd.class_value) if (self.is_classification and not self.is_one_vs_all) \
                        else (nd.predict or 0.0)
                    p[i] += val * t.learning_rate
                wsum += t.learning_rate
            if is_gbt:
                p = convert_gbt_score(p, convert)
            else:
                p = p / max(wsum, 1e-300)
            out += p
        return out / max(1, len(self.bags))


def convert_gbt_score(p: np.ndarray, strategy: str) -> np.ndarray:
    """GBT score conversion strategies (IndependentTreeModel :480-514, EvalConfig.gbtScoreConvertStrategy)."""
    s = (strategy or "RAW").upper()
    if s == "OLD_SIGMOID":
        return 1.0 / (1.0 + np.minimum(1e19, np.exp(-p)))
    if s == "SIGMOID":
        return 1.0 / (1.0 + np.minimum(1e19, np.exp(-20 * p)))
    if s in ("CUTOFF", "HALF_CUTOFF"):
        return np.clip(p, 0.0, 1.0)
    if s == "MAXMIN_SCALE":
        lo, hi = p.min(), p.max()
        return (p - lo) / (hi - lo) if hi > lo else np.zeros_like(p)
    return p


# ---- serialization --------------------------------------------------------------------------
def _write_bitset(o: JavaOut, cats: set):
    n = (max(cats) // 8 + 1) if cats else 1
    words = bytearray(max(1, n))
    for c in cats or []:
        words[c >> 3] |= (1 << (c % 8))
    o.int(len(words))
    o.raw(bytes(words))


def _read_bitset(i: JavaIn) -> set:
    n = i.int()
    words = i._take(n)
    return {b * 8 + k for b in range(n) for k in range(8) if (words[b] >> k) & 1}


def _write_node(o: JavaOut, nd: Node):
    o.int(nd.id)
    o.float(nd.gain)
    o.double(nd.wgt_cnt)
    if nd.split is None:
        o.bool(False)
    else:
        o.bool(True)
        s = nd.split
        o.int(s.column)
        o.byte(s.ftype)
        if s.ftype == CATEGORICAL:
            o.bool(s.is_left)
            if s.categories is None:
                o.bool(True)
            else:
                o.bool(False)
                _write_bitset(o, s.categories)
        else:
            o.double(s.threshold)
    real_leaf = nd.is_leaf()
    o.bool(real_leaf)
    if real_leaf:
        if nd.predict is None:
            o.bool(False)
        else:
            o.bool(True)
            o.double(nd.predict)
            o.byte(nd.class_value)
    for ch in (nd.left, nd.right):
        if ch is None:
            o.bool(False)
        else:
            o.bool(True)
            _write_node(o, ch)


def _read_node(i: JavaIn, version: int) -> Node:
    nd = Node(i.int())
    nd.gain = i.float()
    nd.wgt_cnt = i.float() if version <= 2 else i.double()
    if i.bool():
        col = i.int()
        ft = i.byte()
        if ft == CATEGORICAL:
            is_left = i.bool()
            cats = None if i.bool() else _read_bitset(i)
            nd.split = Split(col, ft, 0.0, is_left, cats)
        else:
            nd.split = Split(col, ft, i.double())
    if i.bool():               # isRealLeaf
        if i.bool():
            nd.predict = i.double()
            nd.class_value = i.byte()
    if i.bool():
        nd.left = _read_node(i, version)
    if i.bool():
        nd.right = _read_node(i, version)
    return nd


def write_tree_model(path: str, m: TreeModelFile):
    o = JavaOut()
    o.int(TREE_FORMAT_VERSION)
    o.utf(m.algorithm)
    o.utf(m.loss)
    o.bool(m.is_classification)
    o.bool(m.is_one_vs_all)
    o.int(m.input_count)
    o.int(len(m.numerical_means))
    for k, v in m.numerical_means.items():
        o.int(k)
        o.double(0.0 if v is None else v)
    o.int(len(m.names))
    for k, v in m.names.items():
        o.int(k)
        o.utf(v)
    o.int(len(m.categories))
    for k, cats in m.categories.items():
        o.int(k)
        o.int(len(cats))
        for c in cats:
            if len(c) < MAX_CATEGORICAL_VAL_LEN:
                o.utf(c)
            else:
                o.short(UTF_BYTES_MARKER)
                bs = c.encode("utf-8")
                o.int(len(bs))
                o.raw(bs)
    o.int(len(m.column_mapping))
    for k, v in m.column_mapping.items():
        o.int(k)
        o.int(v)
    write_bags(o, m.bags)
    with open(path, "wb") as f:
        f.write(o.gzip_bytes())


def write_bags(o: JavaOut, bags):
    """int #bags, then per bag int #trees and ``TreeNode.write`` records (the ``.gbt`` tail and
    the ``trees`` entry of the readable zip spec, IndependentTreeModelUtils.java:52-60)."""
    o.int(len(bags))
    for bag in bags:
        o.int(len(bag))
        for t in bag:
            o.int(t.tree_id)
            o.int(t.node_num)
            _write_node(o, t.root)
            o.double(t.learning_rate)
            if t.root.id == 1:
                o.double(t.root_wgt_cnt)
            o.int(len(t.features))
            for f in t.features:
                o.int(f)


def read_bags(i: JavaIn, version: int = TREE_FORMAT_VERSION, n_bags: int | None = None):
    bags = []
    nb = i.int() if n_bags is None else n_bags
    for _ in range(nb):
        trees = []
        for _ in range(i.int()):
            tid = i.int()
            nn = i.int()
            root = _read_node(i, version)
            lr = i.double()
            rw = i.double() if root.id == 1 else 0.0
            feats = [i.int() for _ in range(i.int())]
            trees.append(TreeRecord(tid, nn, root, lr, rw, feats))
        bags.append(trees)
    return bags


def _is_legacy(data: bytes) -> bool:
    """Pre-versioned files start with the int-framed algorithm name ("GBT"/"RF") instead of a
    version int followed by a readUTF string."""
    if len(data) < 8 or data[:2] == b"\x1f\x8b":
        return False
    n = int.from_bytes(data[:4], "big")
    return n in (2, 3) and data[4:4 + n] in (b"GBT", b"RF")


def read_legacy_tree_model(data: bytes) -> TreeModelFile:
    """Legacy (pre-versioned) tree model layout:

      header : String algorithm, double learningRate, String loss, bool isClassification,
               bool isOneVsAll, int treeNum
      tree   : int treeId, int nodeNum, Node root, double rootWgtCnt, int nFeatures, int[] features
      Node   : int id, double gain, double impurity, bool isLeaf, double wgtCntRatio,
               bool hasSplit [Split], bool hasPredict [double predict, double classValue],
               bool hasLeft [Node], bool hasRight [Node]
      Split  : int columnNum, double threshold, String columnName, bool isLeft, UTF featureType
               ("CONTINUOUS"/"CATEGORICAL"), int nCategories, String[] categories
    (String = int byte length + UTF-8 bytes.)  Category strings become per-column category lists so
    the model scores through the same ``TreeModelFile`` path as v4 files."""
    i = JavaIn(bytes(data))

    def jstr():
        n = i.int()
        return i._take(n).decode("utf-8") if n > 0 else ""

    alg = jstr()
    lr = i.double()
    loss = jstr()
    is_cls = i.bool()
    ova = i.bool()
    names, cats = {}, {}

    def node():
        nd = Node(i.int())
        nd.gain = i.double()
        i.double()                       # impurity
        i.bool()                         # isLeaf (derivable from the children)
        nd.wgt_cnt = i.double()          # weight-count ratio of the parent
        if i.bool():
            col = i.int()
            thr = i.double()
            names.setdefault(col, jstr())
            is_left = i.bool()
            ftype = i.utf()
            ncat = i.int()
            vals = [jstr() for _ in range(ncat)]
            if ftype.upper().startswith("CAT"):
                lst = cats.setdefault(col, [])
                idx = set()
                for v in vals:
                    if v not in lst:
                        lst.append(v)
                    idx.add(lst.index(v))
                nd.split = Split(col, CATEGORICAL, 0.0, is_left, idx)
            else:
                nd.split = Split(col, CONTINUOUS, thr, is_left)
        if i.bool():
            nd.predict = i.double()
            nd.class_value = int(i.double())
        if i.bool():
            nd.left = node()
        if i.bool():
            nd.right = node()
        return nd

    trees = []
    for _ in range(i.int()):
        tid = i.int()
        nn = i.int()
        root = node()
        rw = i.double()
        feats = [i.int() for _ in range(i.int())]
        trees.append(TreeRecord(tid, nn, root, lr, rw, feats))
    cols = sorted({f for t in trees for f in t.features} | set(names))
    mapping = {c: j for j, c in enumerate(cols)}
    return TreeModelFile(alg, loss, is_cls, ova, len(cols), {}, names, cats, mapping, [trees], 0)


def iter_nodes(root):
    """Pre-order walk over a record tree."""
    stack = [root] if root is not None else []
    while stack:
        nd = stack.pop()
        yield nd
        if not nd.is_leaf():
            stack.append(nd.right)
            stack.append(nd.left)


def read_tree_model(path_or_bytes) -> TreeModelFile:
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    if _is_legacy(bytes(data)):
        return read_legacy_tree_model(bytes(data))
    i = JavaIn(bytes(data))
    version = i.int()
    alg = i.utf()
    loss = i.utf()
    is_cls = i.bool()
    ova = i.bool()
    inputs = i.int()
    means = {}
    for _ in range(i.int()):
        k = i.int()
        means[k] = i.double()
    names = {}
    for _ in range(i.int()):
        k = i.int()
        names[k] = i.utf()
    cats = {}
    for _ in range(i.int()):
        k = i.int()
        lst = []
        for _ in range(i.int()):
            ml = i.short()
            if ml < 0:
                lst.append(i._take(i.int()).decode("utf-8"))
            else:
                from .javaio import decode_modified_utf8
                lst.append(decode_modified_utf8(i._take(ml)))
        cats[k] = lst
    mapping = {}
    for _ in range(i.int()):
        k = i.int()
        mapping[k] = i.int()
    bags = read_bags(i, version, 1 if version < 4 else None)
    return TreeModelFile(alg, loss, is_cls, ova, inputs, means, names, cats, mapping, bags, version)


# ---- conversion from the GPU trainer's heap trees --------------------------------------------------
def heap_tree_to_record(tree, tree_id: int, columns, ccs_by_feature=None, learning_rate=None,
                        is_classification=False) -> TreeRecord:
    """``models.gbdt.Tree`` (bin thresholds, feature positions) -> TreeRecord with raw-value
    thresholds (``binBoundary[thr+1]``) and column numbers (``Split`` semantics)."""
    def build(nid):
        if nid >= tree.max_nodes or not tree.exists[nid]:
            return None
        nd = Node(int(nid), float(tree.gain[nid]), float(tree.wgt_cnt[nid]))
        f = int(tree.feat[nid])
        if f >= 0:
            cc = columns[f]
            if cc.is_categorical():
                bits = tree.cat_left[nid]
                ncat = len(cc.bin_category or [])
                left = {b for b in range(ncat + 1) if (int(bits[b >> 5]) >> (b & 31)) & 1}
                if ncat + 1 <= len(left) * 2:   # store the smaller side (Impurity.java:171-198)
                    nd.split = Split(cc.num, CATEGORICAL, 0.0, False, set(range(ncat + 1)) - left)
                else:
                    nd.split = Split(cc.num, CATEGORICAL, 0.0, True, left)
            else:
                bb = cc.bin_boundary
                thr = int(tree.thr[nid])
                nd.split = Split(cc.num, CONTINUOUS, float(bb[thr + 1]) if thr + 1 < len(bb) else float("inf"))
            nd.left = build(2 * nid)
            nd.right = build(2 * nid + 1)
        else:
            nd.predict = float(tree.value[nid])
            if getattr(tree, "classification", False):      # native multi-class RF leaf
                nd.class_value = int(tree.class_value[nid])
            else:
                nd.class_value = int(round(tree.value[nid])) if is_classification else 0
        return nd
    root = build(1)
    lr = tree.weight if learning_rate is None else learning_rate
    return TreeRecord(tree_id, int(tree.n_nodes()), root, float(lr), float(tree.wgt_cnt[1]),
                      sorted({columns[f].num for f in tree.features_used}))


def record_to_heap_tree(rec: TreeRecord, columns, min_depth: int = 1):
    """Inverse of ``heap_tree_to_record`` for continuous training: a stored tree (column numbers,
    raw-value thresholds) -> ``models.gbdt.Tree`` over the current binned features.  Node ids are
    heap ids in both (``Node.leftIndex`` = 2 id).  A numeric threshold t maps to the last bin whose
    upper boundary is <= t (exact when the ColumnConfig boundaries are the ones the model was
    trained with); a categorical split's stored side maps to the left-bin bitset."""
    from ..models.gbdt import Tree
    pos = {c.num: j for j, c in enumerate(columns)}

    def max_id(nd):
        return 0 if nd is None else max(nd.id, max_id(nd.left), max_id(nd.right))
    depth = max(min_depth, int(max_id(rec.root)).bit_length())
    t = Tree(depth, float(rec.learning_rate))
    used = set()

    def put(nd):
        if nd is None:
            return
        i = nd.id
        t.exists[i] = True
        t.gain[i] = nd.gain
        t.wgt_cnt[i] = nd.wgt_cnt
        s = nd.split
        if s is not None and not (nd.left is None and nd.right is None) and s.column in pos:
            f = pos[s.column]
            cc = columns[f]
            t.feat[i] = f
            used.add(f)
            if s.ftype == CATEGORICAL:
                ncat = len(cc.bin_category or [])
                stored = set(s.categories or set())
                left = stored if s.is_left else set(range(ncat + 1)) - stored
                for b in left:
                    t.cat_left[i, b >> 5] |= np.uint32(1 << (b & 31))
            else:
                bb = np.asarray(cc.bin_boundary, dtype=np.float64)
                thr = s.threshold
                t.thr[i] = len(bb) - 1 if not np.isfinite(thr) else int(np.searchsorted(bb, thr, "right")) - 2
            put(nd.left)
            put(nd.right)
        else:
            t.value[i] = float(nd.predict or 0.0)
    put(rec.root)
    t.features_used = sorted(used)
    return t


def feature_importance(model: TreeModelFile) -> dict:
    """Gain-accumulated feature importance (TreeNode.computeFeatureImportance, scikit-learn style)."""
    imp = {}

    def walk(nd: Node, total: float):
        if nd is None or nd.split is None or nd.left is None or nd.right is None:
            return
        g = nd.gain * nd.wgt_cnt / max(total, 1e-300)
        imp[nd.split.column] = imp.get(nd.split.column, 0.0) + g
        walk(nd.left, total)
        walk(nd.right, total)
    for bag in model.bags:
        for t in bag:
            walk(t.root, t.root.wgt_cnt or 1.0)
    s = sum(imp.values())
    return {k: v / s for k, v in sorted(imp.items(), key=lambda kv: -kv[1])} if s > 0 else imp
