"""Vectorized tree-ensemble inference on raw values (I2/I6, K13) and leaf encoding (H17).

``IndependentTreeModel.computeRegressionScore`` (J/core/dtrain/dt/IndependentTreeModel.java:387-441)
walks every tree per row.  Here every bag is flattened once into structure-of-arrays node tables
(feature slot, threshold, categorical left-set LUT, children, leaf value).  On the CPU all (row,
tree) pairs descend one level per step as torch gathers (the oracle); on the GPU the HIP kernels
of ``ops/csrc/scoring_kernels.hip`` rank every input against the ensemble's thresholds (u16
codes), stage the rows' codes in LDS and walk all trees per row there (``_hip_walk``).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..formats.tree_format import CONTINUOUS, TreeModelFile, convert_gbt_score

# GPU walk over u16 threshold-rank codes staged in LDS (SHIFU_TREE_CODED=0: fp64 input walk)
CODED_WALK = os.environ.get("SHIFU_TREE_CODED", "1") != "0"


class FlatEnsemble:
    def __init__(self, model: TreeModelFile, bag: int, columns: list, device="cpu"):
        self.model = model
        self.columns = columns                     # column numbers -> input slot order
        slot = {c: i for i, c in enumerate(columns)}
        trees = model.bags[bag]
        feat, thr, iscat, left, right, value, lr_, catrow, roots, depth = [], [], [], [], [], [], [], [], [], 0
        cat_sets, paths = [], []
        max_cat = max([len(v) for v in model.categories.values()] + [0]) + 1
        for t in trees:
            roots.append(len(feat))
            # BFS assigning indices
            order, queue = [], [(t.root, 0, "")]
            while queue:
                nd, d, path = queue.pop(0)
                depth = max(depth, d)
                order.append(nd)
                paths.append(path)
                if not nd.is_leaf():
                    queue.append((nd.left, d + 1, path + "L"))
                    queue.append((nd.right, d + 1, path + "R"))
            base = len(feat)
            idx = {id(nd): base + i for i, nd in enumerate(order)}
            for nd in order:
                if nd.is_leaf():
                    feat.append(-1); thr.append(0.0); iscat.append(0); left.append(idx[id(nd)])
                    right.append(idx[id(nd)])
                    val = float(nd.class_value) if (model.is_classification and not model.is_one_vs_all) \
                        else float(nd.predict or 0.0)
                    value.append(val); catrow.append(-1)
                else:
                    s = nd.split
                    feat.append(slot[s.column]); left.append(idx[id(nd.left)]); right.append(idx[id(nd.right)])
                    value.append(0.0)
                    if s.ftype == CONTINUOUS:
                        thr.append(float(s.threshold)); iscat.append(0); catrow.append(-1)
                    else:
                        thr.append(float(len(model.categories.get(s.column, []))))
                        iscat.append(1)
                        row = np.zeros(max_cat + 1, dtype=bool)
                        cats = s.categories or set()
                        for c in cats:
                            if 0 <= c <= max_cat:
                                row[c] = True
                        if not s.is_left:          # stored set is the right side
                            row = ~row
                        catrow.append(len(cat_sets)); cat_sets.append(row)
            lr_.append(float(t.learning_rate))
        dev = torch.device(device)
        self.dev = dev
        self.depth = depth
        self.feat = torch.tensor(feat, dtype=torch.int64, device=dev)
        self.thr = torch.tensor(thr, dtype=torch.float64, device=dev)
        self.iscat = torch.tensor(iscat, dtype=torch.bool, device=dev)
        self.left = torch.tensor(left, dtype=torch.int64, device=dev)
        self.right = torch.tensor(right, dtype=torch.int64, device=dev)
        self.value = torch.tensor(value, dtype=torch.float64, device=dev)
        self.catrow = torch.tensor(catrow, dtype=torch.int64, device=dev)
        self.catlut = torch.from_numpy(np.stack(cat_sets) if cat_sets else np.zeros((1, max_cat + 1), bool)).to(dev)
        self.max_cat = max_cat
        self.roots = torch.tensor(roots, dtype=torch.int64, device=dev)
        self.lrs = torch.tensor(lr_, dtype=torch.float64, device=dev)
        self.paths = np.array(paths, dtype=object)     # L/R path from the root of every node

    # ---- HIP path (K13: scoring_kernels.hip tree_infer_kernel) ----------------------------
    def _hip_tables(self):
        if getattr(self, "_ht", None) is None:
            node = torch.stack([self.feat, self.left, self.right,
                                torch.where(self.iscat, self.catrow, torch.full_like(self.catrow, -1))], 1)
            self._ht = (node.to(torch.int32).contiguous(), self.thr.contiguous(), self.value.contiguous(),
                        self.catlut.to(torch.uint8).contiguous(), self.roots.to(torch.int32).contiguous(),
                        self.lrs.contiguous())
        return self._ht

    def _coded_tables(self, C: int):
        """Tables of the coded walk (scoring_kernels.hip tree_code / tree_walk_coded): per input
        slot the sorted unique thresholds the ensemble compares it with, node records whose 4th
        field is the threshold's rank (numeric: left iff code <= rank) or -(LUT row + 1)
        (categorical), and the category count per LUT row.  None when the coded walk cannot hold
        the ensemble (> 65534 thresholds on one feature, or > 16384 inputs)."""
        if getattr(self, "_ct", None) is not None or getattr(self, "_ct_none", False):
            return self._ct
        feat, thr = self.feat.cpu().numpy(), self.thr.cpu().numpy()
        iscat, catrow = self.iscat.cpu().numpy(), self.catrow.cpu().numpy()
        num = (feat >= 0) & ~iscat
        order = np.lexsort((thr[num], feat[num]))
        fs, ts = feat[num][order], thr[num][order]
        keep = np.ones(len(fs), bool)
        keep[1:] = (fs[1:] != fs[:-1]) | (ts[1:] != ts[:-1])
        fs, ts = fs[keep], ts[keep]
        boff = np.searchsorted(fs, np.arange(C + 1), side="left").astype(np.int32)
        if C > 16384 or (len(boff) > 1 and np.diff(boff).max(initial=0) >= 65535):
            self._ct_none = True
            return None
        w = np.zeros(len(feat), np.int64)
        ni = np.nonzero(num)[0]
        for f in np.unique(feat[ni]):                  # one vectorized search per feature
            idx = ni[feat[ni] == f]
            w[idx] = np.searchsorted(ts[boff[f]:boff[f + 1]], thr[idx], side="left")
        cat = (feat >= 0) & iscat
        w[cat] = -(catrow[cat] + 1)
        n_catrows = int(self.catlut.shape[0])
        catnc = np.zeros(max(1, n_catrows), np.int32)
        catnc[catrow[cat]] = thr[cat].astype(np.int64)
        slot_cat = np.array([c in self.model.categories for c in self.columns], np.uint8)
        dev = self.dev
        node = torch.from_numpy(np.stack([feat, self.left.cpu().numpy(), self.right.cpu().numpy(), w], 1)
                                .astype(np.int32)).to(dev)
        tiles = np.minimum(np.arange(0, C + 32, 32), C)         # 32-feature tiles of the code kernel
        tb_cap = int(np.diff(boff[np.unique(tiles)]).max(initial=0))
        self._ct = (torch.from_numpy(ts.astype(np.float64) if len(ts) else np.zeros(1)).to(dev),
                    torch.from_numpy(boff).to(dev), torch.from_numpy(slot_cat).to(dev), node,
                    torch.from_numpy(catnc).to(dev), tb_cap)
        return self._ct

    def _hip_walk(self, X: torch.Tensor, want_leaves: bool):
        """One kernel launch for all (row, tree) pairs of the chunk: -> (bag score, leaf ids | None)."""
        from ..ops import _native
        _native.require_gpu_native()
        n, T = X.shape[0], int(self.roots.numel())
        XT = X.to(torch.float64).t().contiguous()             # feature-major [C, N]: coalesced at the root
        C = XT.shape[0]
        node, thr, value, lut, roots, lrs = self._hip_tables()
        ct = self._coded_tables(C) if CODED_WALK else None
        if ct is not None:
            bnd, boff, slot_cat, cnode, catnc, tb_cap = ct
            R = 1 << max(0, min(8, int(np.floor(np.log2(16384 / max(C, 1))))))
            rb = -(-n // R)
            groups = max(1, min(T, -(-2048 // rb)))
            groups = -(-T // -(-T // groups))
            part = torch.empty(groups, n, dtype=torch.float64, device=X.device)
            leaf = torch.empty(n, T, dtype=torch.int32, device=X.device) if want_leaves else None
            step = min(65535 * 256, max(1, (1 << 31) // max(C, 1) // 2))   # codes chunk <= 2 GiB
            codes = torch.empty(min(n, step), C, dtype=torch.int16, device=X.device)
            for r0 in range(0, n, step):
                m = min(n, r0 + step) - r0
                # pointer offsets into the full-width buffers: no per-chunk copies
                _native.call_hip("shifu_tree_code", XT.data_ptr() + r0 * 8, n, m, C, bnd, boff, slot_cat, codes,
                                 tb_cap, _native.stream_of(X))
                lv = None if leaf is None else leaf.data_ptr() + r0 * T * 4
                _native.call_hip("shifu_tree_walk_coded", codes, m, C, cnode, catnc, value, lut, lut.shape[1],
                                 roots, lrs, T, max(self.depth, 0), R, groups, part.data_ptr() + r0 * 8, n, lv,
                                 _native.stream_of(X))
            return part.sum(0), leaf
        groups = max(1, min(T, -(-2048 // max(1, -(-n // 256)))))
        groups = -(-T // -(-T // groups))                     # every group owns >= 1 tree
        part = torch.empty(groups, n, dtype=torch.float64, device=X.device)
        leaf = torch.empty(n, T, dtype=torch.int32, device=X.device) if want_leaves else None
        _native.call_hip("shifu_tree_infer", XT, n, 1, n, node, thr, value, lut, lut.shape[1], roots, lrs, T,
                         max(self.depth, 0), groups, part, leaf, _native.stream_of(X))
        return part.sum(0), leaf

    @torch.no_grad()
    def leaves(self, X: torch.Tensor) -> torch.Tensor:
        """X [N, C] float64 (numeric raw values, categorical indices) -> leaf node ids [N, T]."""
        if X.is_cuda and X.shape[0] and self.roots.numel():
            return self._hip_walk(X, True)[1].long()
        n = X.shape[0]
        node = self.roots.unsqueeze(0).expand(n, -1).clone()
        rows = torch.arange(n, device=self.dev).unsqueeze(1)
        for _ in range(self.depth):
            f = self.feat[node]
            inner = f >= 0
            v = X[rows.expand_as(node), f.clamp(min=0)]
            cat = self.iscat[node]
            go_left = v < self.thr[node]
            if bool(cat.any()):
                nc = self.thr[node]
                ci = torch.where((v < 0) | (v >= nc), nc, torch.floor(v + 0.1)).long().clamp(0, self.max_cat)
                inset = self.catlut[self.catrow[node].clamp(min=0), ci]
                go_left = torch.where(cat, inset, go_left)
            nxt = torch.where(go_left, self.left[node], self.right[node])
            node = torch.where(inner, nxt, node)
        return node

    @torch.no_grad()
    def score(self, X: torch.Tensor) -> torch.Tensor:
        """Bag score: GBT -> sum lr*leaf (raw), RF -> weighted mean of leaves."""
        if X.is_cuda and X.shape[0] and self.roots.numel():
            s = self._hip_walk(X, False)[0]
        else:
            lv = self.value[self.leaves(X)]                   # [N, T]
            s = (lv * self.lrs).sum(1)
        if self.model.algorithm.upper() != "GBT":
            s = s / self.lrs.sum().clamp(min=1e-300)
        return s


class TreeScorer:
    """Raw-row scorer for a whole ``.gbt``/``.rf`` file (all bags, averaged)."""

    def __init__(self, model: TreeModelFile, device="cpu", convert: str = "RAW"):
        self.model = model
        self.columns = sorted(model.names.keys())
        self.ens = [FlatEnsemble(model, b, self.columns, device) for b in range(len(model.bags))]
        self.dev = torch.device(device)
        self.convert = convert

    def input_matrix(self, table) -> torch.Tensor:
        """RawTable (or {name: raw values}) -> [N, C] float64 via ``TreeModelFile.vectorize`` rules."""
        m = self.model
        n = table.n if hasattr(table, "n") else len(next(iter(table.values())))
        X = np.empty((n, len(self.columns)), dtype=np.float64)
        for j, c in enumerate(self.columns):
            name = m.names[c]
            col = table[name]
            if c in m.categories:
                cats = m.categories[c]
                lut = {}
                for i, cv in enumerate(cats):
                    for sv in str(cv).split("^"):
                        lut.setdefault(sv, i)
                if hasattr(col, "kind") and col.kind == "str":
                    mp = np.array([lut.get(s, len(cats)) for s in col.dictionary] + [len(cats)], dtype=np.float64)
                    X[:, j] = mp[np.where(col.values >= 0, col.values, len(col.dictionary))]
                else:
                    strs = col.strings() if hasattr(col, "strings") else [str(v) for v in col]
                    X[:, j] = [lut.get(s, len(cats)) for s in strs]
            else:
                v = col.numeric().astype(np.float64) if hasattr(col, "numeric") else \
                    np.array([_to_float(x) for x in col])
                X[:, j] = np.where(np.isnan(v), m.numerical_means.get(c, 0.0), v)
        return torch.from_numpy(X).to(self.dev)

    @torch.no_grad()
    def score_bags(self, X: torch.Tensor, chunk: int | None = None) -> np.ndarray:
        chunk = chunk or ((1 << 20) if X.is_cuda else (1 << 16))
        out = []
        for e in self.ens:
            parts = [e.score(X[i: i + chunk]) for i in range(0, X.shape[0], chunk)]
            s = torch.cat(parts).cpu().numpy() if parts else np.zeros(0)
            if self.model.algorithm.upper() == "GBT":
                s = convert_gbt_score(s, self.convert)
            out.append(s)
        return np.stack(out, 1) if out else np.zeros((X.shape[0], 0))

    def score(self, table) -> np.ndarray:
        return self.score_bags(self.input_matrix(table)).mean(1)

    def class_votes(self, table, n_classes: int, chunk: int = 1 << 16) -> np.ndarray:
        """Native multi-class forests (classification leaves carry a class value): per row the
        fraction of trees voting for each class, averaged over bags -> [N, n_classes]
        (``computeClassificationScore`` returns every tree's class; the caller votes)."""
        X = self.input_matrix(table)
        out = np.zeros((X.shape[0], n_classes))
        for e in self.ens:
            for i in range(0, X.shape[0], chunk):
                lv = e.value[e.leaves(X[i: i + chunk])].round().long().clamp(0, n_classes - 1)
                cnt = torch.zeros(lv.shape[0], n_classes, dtype=torch.float64, device=lv.device)
                cnt.scatter_add_(1, lv, torch.ones_like(lv, dtype=torch.float64))
                out[i: i + chunk] += (cnt / max(lv.shape[1], 1)).cpu().numpy()
        return out / max(len(self.ens), 1)

    @torch.no_grad()
    def encode(self, table, depth: int | None = None) -> np.ndarray:
        """Leaf-path encoding (``IndependentTreeModel.encode`` J/core/dtrain/dt/IndependentTreeModel.java:272-350):
        per tree the L/R path to the reached leaf, right-padded with "L" to ``depth`` characters
        -> [N, total trees] strings usable as categorical features of a downstream model."""
        X = self.input_matrix(table)
        cols = []
        for e in self.ens:
            d = depth or max(1, e.depth)
            leaf = e.leaves(X).cpu().numpy()
            pad = np.vectorize(lambda p: (p + "L" * d)[:d], otypes=[object])
            cols.append(pad(e.paths[leaf]))
        return np.concatenate(cols, 1) if cols else np.zeros((X.shape[0], 0), dtype=object)

    @torch.no_grad()
    def encode_fields(self, table, depth: int | None = None) -> list:
        """:meth:`encode` as row-formatter fields (data/join.py): per tree (DICT, int32 code per
        row, padded paths of the leaves reached) -- no per-row Python strings.  The leaf walk runs
        on the scorer's device (HIP tree walk on a GPU)."""
        from ..data.join import DICT
        X = self.input_matrix(table)
        out = []
        for e in self.ens:
            d = depth or max(1, e.depth)
            leaf = e.leaves(X).cpu().numpy()
            for t in range(leaf.shape[1]):
                u, inv = np.unique(leaf[:, t], return_inverse=True)
                out.append((DICT, inv.astype(np.int32), [(p + "L" * d)[:d] for p in e.paths[u]]))
        return out


def _to_float(x):
    try:
        return float(x)
    except (TypeError, ValueError):
        return float("nan")
