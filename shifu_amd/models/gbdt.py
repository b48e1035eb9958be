"""Gradient-boosted trees (GBT) and random forest (RF) on MI355X.

Reference behaviour (Shifu ``GBT``/``RF``):
  * rows are binned (``DTWorker.getBinIndex`` J/core/dtrain/dt/DTWorker.java:1001-1034);
    categorical missing/unknown -> last bin (``:1148-1170``).
  * level-wise growth to ``MaxDepth`` (root = level 1; children at level MaxDepth are leaves,
    ``DTMaster.splitNodeForLevelWisedTree`` J/core/dtrain/dt/DTMaster.java:566-605).
  * split search per (node, feature) = prefix scan over bins with ``MinInstancesPerNode`` /
    ``MinInfoGain`` (``Impurity.computeImpurity`` J/core/dtrain/dt/Impurity.java:120-211);
    categorical bins are ordered by mean target first.  Feature subsets are drawn per node
    (``DTMaster.getSubsamplingFeatures`` :822-850).
  * GBT: first tree fits the label and sets predict = leaf (weight 1.0); later trees fit
    -dLoss/dpredict and add learningRate * leaf (``DTWorker.doCompute`` :620-670, ``Loss.java``).
    Leaf value = weighted mean of the node's targets (no Newton step).
  * RF: per-tree bagging weights (Poisson with replacement / Bernoulli), score = mean of trees.

MI355X design: see ``ops/csrc/gbdt_kernels.hip`` (LDS histogram per (node, row range,
32-feature group) work item, slab reduce + sibling subtraction + split scan, stable
partition of a position->row permutation, tree application).  Multi-GPU: each rank owns a
row shard; built-node histograms are all-reduced over RCCL (one bucket per level) and the
split search is replicated deterministically, so no trees are ever broadcast.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..parallel import dist
from ..utils.log import get_logger
from ..utils.trace import trace_range

_log = get_logger("models.gbdt")

NB = 256
FG = 32                     # features per histogram work-item group (gbdt_kernels.hip FG)
QF = 128                    # features per 128-B row record of the quad-blocked bins (QF)
IMPURITY_IDS = {"variance": 0, "friedmanmse": 1, "entropy": 2, "gini": 3}
LOSS_IDS = {"squared": 0, "halfgradsquared": 1, "absolute": 2, "log": 3}


# histogram work items per level (node x row-range x 32-feature group); SHIFU_GBDT_ITEMS: lab A/B
TARGET_ITEMS = int(os.environ.get("SHIFU_GBDT_ITEMS", "4096"))   # favourable +2.3 %, balanced even vs 2048 (profiles/r5/gbdt/items_sweep_r5.txt)
TARGET_ITEMS_FEW = int(os.environ.get("SHIFU_GBDT_ITEMS_FEW", str(TARGET_ITEMS // 2)))   # non-root levels, <= 4 built nodes


def _strategy_count(strategy, n_feat: int, input_num: int, tree_num: int) -> int:
    """Number of features a node samples (DTMaster.getSubsamplingFeatures); 0 = all."""
    if strategy is None:
        return n_feat
    if isinstance(strategy, (int, float)) and not isinstance(strategy, bool):
        return max(1, int(n_feat * float(strategy)))
    s = str(strategy).strip().upper()
    try:
        v = float(s)
        return max(1, int(n_feat * v))
    except ValueError:
        pass
    if s == "HALF":
        return n_feat // 2
    if s == "ONETHIRD":
        return n_feat // 3
    if s == "TWOTHIRDS":
        return n_feat * 2 // 3
    if s == "SQRT":
        return int(n_feat * math.sqrt(input_num) / input_num)
    if s == "LOG2":
        return int(n_feat * math.log(input_num) / math.log(2) / input_num)
    if s == "AUTO":
        return n_feat // 2 if tree_num > 1 else n_feat
    return n_feat


def _h2d(a, dev):
    """Host array -> device tensor through pinned memory with a non-blocking copy: a pageable
    ``.to(device)`` waits for every kernel queued on the stream, so the per-level bookkeeping
    arrays of the tree builder would drain the GPU pipeline a dozen times per level."""
    t = torch.as_tensor(np.ascontiguousarray(a))
    if torch.device(dev).type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


@dataclass
class TreeConfig:
    algorithm: str = "GBT"              # GBT | RF
    tree_num: int = 100
    max_depth: int = 7
    min_instances_per_node: int = 5
    min_info_gain: float = 0.0
    impurity: str = "variance"
    loss: str = "squared"
    learning_rate: float = 0.05
    feature_subset_strategy: object = "TWOTHIRDS"
    bagging_sample_rate: float = 1.0
    sample_with_replacement: bool = False
    dropout_rate: float = 0.0
    max_leaves: int = 0                 # > 0: leaf budget, best (gain x weight) splits first
    max_batch_split: int = 0            # MaxBatchSplitSize: leaf-wise nodes split per level (0 = no cap)
    max_stats_memory_mb: int = 0        # MaxStatsMemoryMB: node-batch bound of the reference (DTMaster
                                        # :437-476); every level's histograms fit in HBM, so it only logs
    seed: int = 0
    valid_tolerance: float = 0.0
    early_stop: bool = False
    n_classes: int = 0                  # RF classification with Entropy/Gini over > 2 classes: native
                                        # multi-class trees (per-class bin stats, Impurity.java:368-734)

    def __post_init__(self):
        self.algorithm = self.algorithm.upper()
        self.impurity = (self.impurity or "variance").lower()
        if self.impurity not in IMPURITY_IDS:
            self.impurity = "variance"
        self.loss = (self.loss or "squared").lower()
        if self.loss not in LOSS_IDS:
            self.loss = "squared"

    @property
    def is_gbt(self):
        return self.algorithm == "GBT"

    @property
    def is_multiclass(self):
        return (not self.is_gbt) and self.n_classes > 2 and self.impurity in ("entropy", "gini")


class Tree:
    """Heap-indexed tree (node id 1 = root, children 2i / 2i+1 as ``Node.leftIndex``)."""

    def __init__(self, max_depth: int, weight: float = 1.0):
        self.max_depth = max_depth
        self.max_nodes = 1 << max_depth
        m = self.max_nodes
        self.feat = np.full(m, -1, dtype=np.int32)      # feature index (into the binned matrix)
        self.thr = np.full(m, -1, dtype=np.int32)       # numeric: left iff bin <= thr
        self.cat_left = np.zeros((m, 8), dtype=np.uint32)
        self.value = np.zeros(m, dtype=np.float32)
        self.class_value = np.zeros(m, dtype=np.float32)  # multi-class RF: argmax class per node
        self.classification = False
        self.wgt_cnt = np.zeros(m, dtype=np.float64)
        self.gain = np.zeros(m, dtype=np.float32)
        self.exists = np.zeros(m, dtype=bool)
        self.weight = float(weight)                     # GBT: 1.0 for the first tree, else lr
        self.features_used = []

    def n_nodes(self) -> int:
        return int(self.exists.sum())

    def leaves(self):
        return [i for i in range(1, self.max_nodes) if self.exists[i] and self.feat[i] < 0]

    def device_arrays(self, device, classes: bool = False):
        return (torch.from_numpy(self.feat).to(device), torch.from_numpy(self.thr).to(device),
                torch.from_numpy(self.cat_left.view(np.int32)).to(device),
                torch.from_numpy(self.class_value if classes else self.value).to(device))

    def predict_bins(self, bins: np.ndarray, is_cat: np.ndarray, classes: bool = False) -> np.ndarray:
        """Host traversal (oracle for the HIP apply kernel)."""
        n = bins.shape[0]
        ids = np.ones(n, dtype=np.int64)
        for _ in range(self.max_depth):
            f = self.feat[ids]
            active = f >= 0
            if not active.any():
                break
            fa = np.where(active, f, 0)
            b = bins[np.arange(n), fa].astype(np.int64)
            catm = is_cat[fa].astype(bool)
            bit = (self.cat_left[ids, b >> 5] >> (b & 31).astype(np.uint32)) & 1
            left = np.where(catm, bit == 1, b <= self.thr[ids])
            ids = np.where(active, np.where(left, 2 * ids, 2 * ids + 1), ids)
        return (self.class_value if classes else self.value)[ids]


@dataclass
class BinnedData:
    """Resident binned shard: uint8 codes in the group-blocked layout ``[G, N, 32]`` (32
    features per group, G = ceil(F / 32), padding features code 0) + targets/weights.

    Blocked rather than row-major so the histogram kernel streams each 32-feature group's
    rows as contiguous 32-B records (see ``ops/csrc/gbdt_kernels.hip``)."""
    bins: torch.Tensor
    y: torch.Tensor
    sig: torch.Tensor | None
    nbins: np.ndarray               # [F] bins per feature (numeric: #boundaries, cat: #cats+1)
    is_cat: np.ndarray              # [F] uint8
    n_feat: int
    # out-of-core: bins in pinned host memory, read by the kernels in place over the
    # host link (the device address of the mapping); targets / weights / predictions stay in HBM
    bins_dptr: int | None = None

    @property
    def n(self):
        return self.bins.shape[1]

    @property
    def device(self):
        return self.y.device

    @property
    def kbins(self):
        """What the HIP kernels get for the bins: the HBM tensor, or the device address of the
        pinned host copy."""
        return self.bins if self.bins_dptr is None else self.bins_dptr

    @property
    def group_stride(self) -> int:
        """Bytes between consecutive 128-feature record blocks of the quad-blocked layout."""
        return self.bins.shape[1] * QF

    def codes(self) -> torch.Tensor:
        """Row-major ``[N, F]`` view (a copy) of the codes - CPU paths and tests."""
        q, n, _ = self.bins.shape
        return self.bins.permute(1, 0, 2).reshape(n, q * QF)[:, : self.n_feat]

    @staticmethod
    def host_resident(codes, y, nbins, is_cat=None, sig=None, device="cuda", rows=None):
        """Like :meth:`from_codes` but the blocked bins stay in pinned host memory (tables larger
        than HBM): the kernels read them through the host mapping's device address
        (``hipHostGetDevicePointer``; refused loudly if the runtime cannot map the buffer)."""
        n, f = codes.shape
        if rows is not None:
            n = len(rows)
        b = torch.empty((f + QF - 1) // QF, n, QF, dtype=torch.uint8, pin_memory=True)
        BinnedData.blocked(codes, "cpu", rows, out=b)
        dptr = _host_device_pointer(b)
        d = BinnedData.from_codes(np.zeros((0, f), np.uint8), np.zeros(0), nbins, is_cat, None, device)
        d.bins, d.bins_dptr = b, dptr
        d.y = torch.as_tensor(y, dtype=torch.float32).reshape(n).to(device)
        d.sig = None if sig is None else torch.as_tensor(sig, dtype=torch.float32).reshape(n).to(device)
        return d

    @staticmethod
    def blocked(codes, device="cpu", rows=None, out=None) -> torch.Tensor:
        """Row-major codes [N, F] (torch or numpy incl. a uint8 memmap, any int dtype) -> quad-blocked
        uint8 [Q, N', 128] on ``device`` (128 features of a row = one 128-B record), filled one
        32-feature group at a time (optionally only ``rows``): host memory stays at one group
        slice, never an int32 copy of the whole matrix."""
        n, f = codes.shape
        if rows is not None:
            n = len(rows)
        q = (f + QF - 1) // QF
        b = torch.zeros(q, n, QF, dtype=torch.uint8, device=device) if out is None else out
        if out is not None and f % QF:
            out[-1, :, f % QF:] = 0
        for gi in range((f + FG - 1) // FG):
            c0, c1 = gi * FG, min(f, (gi + 1) * FG)
            blk = codes[:, c0:c1] if rows is None else codes[rows, c0:c1]
            if isinstance(blk, np.ndarray):
                blk = np.ascontiguousarray(blk, dtype=np.uint8)
                if not blk.flags.writeable:        # read-only memmap slice: torch wants writable memory
                    blk = blk.copy()
                blk = torch.from_numpy(blk)
            o = (gi % (QF // FG)) * FG
            b[gi // (QF // FG), :, o: o + c1 - c0] = blk.to(device=device, dtype=torch.uint8)
        return b

    @staticmethod
    def from_codes(codes, y, nbins, is_cat=None, sig=None, device="cpu", rows=None):
        if not isinstance(codes, np.ndarray):
            codes = torch.as_tensor(codes)
        f = codes.shape[1]
        n = codes.shape[0] if rows is None else len(rows)
        b = BinnedData.blocked(codes, device, rows)
        y = torch.as_tensor(y, dtype=torch.float32).reshape(n).to(device)
        s = None if sig is None else torch.as_tensor(sig, dtype=torch.float32).reshape(n).to(device)
        nb = np.asarray(nbins, dtype=np.int32).reshape(f)
        ic = np.zeros(f, np.uint8) if is_cat is None else np.asarray(is_cat, dtype=np.uint8).reshape(f)
        return BinnedData(b, y, s, nb, ic, f)


class TreeTrainer:
    """Level-wise GBT/RF trainer over a resident binned shard."""

    def __init__(self, cfg: TreeConfig, data: BinnedData, valid: BinnedData | None = None,
                 items_per_node_group: int | None = None):
        self.cfg = cfg
        self.data = data
        self.valid = valid
        self.dev = data.device
        self.gpu = self.dev.type == "cuda"
        if self.gpu:
            from ..ops import _native
            _native.require_gpu_native()
        self.F = data.n_feat
        self.ngroups = (self.F + FG - 1) // FG
        self.trees: list[Tree] = []
        self.pred = torch.zeros(data.n, dtype=torch.float32, device=self.dev)
        self.vpred = None if valid is None else torch.zeros(valid.n, dtype=torch.float32, device=valid.device)
        self.nbins_t = _h2d(data.nbins.astype(np.int32), self.dev)
        self.is_cat_t = _h2d(data.is_cat.astype(np.uint8), self.dev)
        self.rng = np.random.default_rng(cfg.seed)
        self.tgen = torch.Generator(device=self.dev).manual_seed(cfg.seed + 17 * dist.info().rank)
        self.n_sub = _strategy_count(cfg.feature_subset_strategy, self.F, self.F, cfg.tree_num)
        if self.n_sub <= 0 or self.n_sub > self.F:
            self.n_sub = self.F
        # work-item sizing: enough items to fill 256 CUs x 2 at the root
        self.items_per_node_group = items_per_node_group
        self.train_errors: list[float] = []
        self.valid_errors: list[float] = []
        self.timings = {"hist": 0.0, "split": 0.0, "partition": 0.0, "apply": 0.0}
        self.level_stats = None        # list -> per-level histogram events (GPU), see bench_rounds
        # always-on phase accounting (DTWorker's per-phase nanoTime logs, DTWorker.java:581-687):
        # rows histogrammed so far, and per tree the level table + histogram all-reduce time
        self.hist_rows_total = 0
        self.last_tree_stats = None
        self._ar_events = []
        self._root_level = False
        self._codes_cache = None
        self._nmod, self._npos = 0, data.n
        self._pending: list = []        # RF trees grown ahead in a forest batch
        self._fuse = None                # (pred, scale): GBT prediction update fused into the partition

    def _codes(self) -> torch.Tensor:
        """Row-major codes for the CPU paths (built once)."""
        if self._codes_cache is None:
            self._codes_cache = self.data.codes()
        return self._codes_cache

    # ------------------------------------------------------------------------------------
    def _reseed_rows(self, tree_index: int) -> None:
        """Row-level randomness (bagging sub-samples, GBT dropout) is a pure function of (seed,
        rank, first tree of the batch): a run resumed from a checkpoint draws exactly the streams
        of an uninterrupted run, and every rank's shard draws its own (uncorrelated) stream."""
        r = dist.info().rank
        self.tgen.manual_seed((self.cfg.seed * 1_000_003 + r * 7_919 + tree_index * 104_729) % (1 << 63))

    def _weights_for_tree(self) -> torch.Tensor:
        return self._subsample()[1]

    def _subsample(self):
        """(per-row bag weight or None when every row is in the bag, sig * bag weight)."""
        c = self.cfg
        n = self.data.n
        if self.data.sig is not None:
            sig = self.data.sig
        else:                  # one persistent tensor: an unchanged weight vector keeps the root cache valid
            if getattr(self, "_unit_w", None) is None or self._unit_w.numel() != n:
                self._unit_w = torch.ones(n, device=self.dev)
            sig = self._unit_w
        rate = c.bagging_sample_rate
        if c.sample_with_replacement or (not c.is_gbt and c.sample_with_replacement):
            sub = torch.poisson(torch.full((n,), rate, device=self.dev), generator=self.tgen)
        elif rate < 1.0:
            sub = (torch.rand(n, device=self.dev, generator=self.tgen) <= rate).float()
        else:
            return None, sig.contiguous()
        return sub, (sig * sub).contiguous()

    def _node_feature_mask(self, n_nodes: int) -> torch.Tensor | None:
        if self.n_sub >= self.F:
            return None
        m = np.zeros((n_nodes, self.F), dtype=np.uint8)
        rngs = getattr(self, "_level_rngs", None) or [self.rng] * n_nodes
        for i in range(n_nodes):
            m[i, rngs[i].choice(self.F, self.n_sub, replace=False)] = 1
        return _h2d(m, self.dev)

    # ------------------------------------------------------------------------------------
    def grow_tree(self, g: torch.Tensor, w: torch.Tensor, weight: float, tid: int | None = None) -> Tree:
        return self.grow_forest(g, [w], weight, [len(self.trees) if tid is None else tid])[0]

    def grow_forest(self, g: torch.Tensor, ws: list, weight: float, tids: list) -> list:
        """Grow ``len(ws)`` trees at the same time (RF tree parallelism, F5: DTWorker keeps a
        per-tree subsample weight per row, J/core/dtrain/dt/DTWorker.java:1515-1575, and the master
        grows every tree's todo nodes together).  Tree t's rows live at virtual positions
        [t*N, (t+1)*N): pos2row holds t*N + row, the weights / targets are concatenated per tree
        and the kernels read bins at (virtual row mod N).  Each level is ONE histogram launch over
        every tree's built nodes and ONE histogram all-reduce.  Feature subsets come from a
        per-tree generator, so a tree is identical whether it grows alone or in a batch."""
        c = self.cfg
        d = self.data
        n = d.n
        T = len(ws)
        P = T * n
        if P >= 2 ** 31:
            raise ValueError("forest batch exceeds int32 positions; lower the batch")
        self._nmod = n if T > 1 else 0
        self._npos = P
        w = ws[0] if T == 1 else torch.cat(ws)
        gg = g if T == 1 else g.repeat(T)
        # single GPU tree: (w, g) travel in position order with pos2row (the partition scatter moves
        # them), so below the root the histogram reads them contiguously and gathers only the bins;
        # at the root positions are rows
        self._wg_pos = (w, gg) if (self.gpu and T == 1 and not c.is_multiclass and WG_POS) else None
        trees = [Tree(c.max_depth, weight) for _ in range(T)]
        rngs = [np.random.default_rng([c.seed, int(t)]) for t in tids]
        pos2row = torch.arange(P, dtype=torch.int32, device=self.dev)
        pos_node = (pos2row // max(1, n)).to(torch.int32) if T > 1 else torch.zeros(n, dtype=torch.int32,
                                                                                        device=self.dev)
        nodes = [{"tree": t, "id": 1, "start": t * n, "end": (t + 1) * n, "built": True, "parent": -1,
                  "sibling": -1} for t in range(T)]
        hist_prev = None
        # root stats for each root's own value (one all-reduce for the batch)
        # fixed-point scales (powers of two, identical on every rank): per row w*scale_w < 2^16 and
        # |w*g*scale_g| < 2^23, the field widths of the packed LDS histogram entries
        if self.gpu:        # one read of (w, g) per tree: sums and maxima in one deterministic kernel
            from ..ops import _native as nat
            part = torch.empty(4 * 1024, dtype=torch.float64, device=self.dev)
            wst = torch.empty(T, 4, dtype=torch.float64, device=self.dev)
            for t, wt in enumerate(ws):
                nat.call_hip("shifu_gbdt_wg_stats", wt, g, n, part, wst[t], nat.stream_of(d.y))
            tot = dist.all_reduce_(wst[:, :2].contiguous())
            mx = torch.stack([wst[:, 2].max(), wst[:, 3].max()])
        else:
            tot = dist.all_reduce_(torch.stack([torch.stack([wt.double().sum(), (wt.double() * g.double()).sum()])
                                                for wt in ws]))
            mx = torch.stack([w.abs().max().double(), (w * gg).abs().max().double()])
        dist.all_reduce_(mx, "max")
        # the root sums and the scales' maxima in one device-to-host copy (one sync per tree here)
        hv = torch.cat([tot.reshape(-1).double(), mx.double()]).cpu().numpy()
        tot, mx = hv[:2 * T].reshape(T, 2), hv[2 * T:]
        self.scale_w = _pack_scale(float(mx[0]), W_BITS)
        # margin 2^(GSH32+1): the root's u32 w*g mode quantises at scale_g / 2^GSH32, whose rounded
        # |q| must stay < 2^20 - 1 so 2048 rows in one bin cannot reach 2^31 (gbdt_kernels.hip)
        self.scale_g = _pack_scale(float(mx[1]), G_BITS, margin=2.0 ** (ROOT_GSH32 + 1))
        for t, tree in enumerate(trees):
            tw, ts = float(tot[t, 0]), float(tot[t, 1])
            tree.exists[1] = True
            tree.value[1] = ts / tw if tw != 0 else 0.0
            tree.wgt_cnt[1] = tw
        if self.cfg.is_multiclass:     # root Predict: P(class 1) and the majority class
            C = self.cfg.n_classes
            yl = g.round().long().clamp(0, C - 1)
            ctot = torch.stack([torch.zeros(C, dtype=torch.float64, device=self.dev).index_add_(0, yl, wt.double())
                                for wt in ws])
            dist.all_reduce_(ctot)
            ctot = ctot.cpu().numpy()
            for t, tree in enumerate(trees):
                sw = ctot[t].sum()
                tree.classification = True
                tree.value[1] = ctot[t, 1] / sw if sw > 0 else 0.0
                tree.class_value[1] = float(np.argmax(ctot[t])) if sw > 0 else 0.0
        n_leaves = [1] * T
        level_log = []
        self.last_tree_stats = {"levels": level_log}
        if self._pipelined(T):
            self._grow_levels_dev(trees, rngs, nodes, pos2row, pos_node, w, gg, level_log, n_leaves)
            self._nmod, self._npos = 0, n
            return trees
        for level in range(1, c.max_depth):
            if not nodes:
                break
            # slots: built nodes first (contiguous for the all-reduce), then derived, by (tree, id);
            # the partition already wrote these slot ids into pos_node (no remap pass)
            nodes.sort(key=_slot_key)
            for s_, z in enumerate(nodes):
                z["slot"] = s_
            slot_of = {(z["tree"], z["id"]): z["slot"] for z in nodes}
            for z in nodes:
                if not z["built"]:
                    z["sib_slot"] = slot_of[(z["tree"], z["id"] ^ 1)]
            n_built = sum(1 for z in nodes if z["built"])
            self._root_level = level == 1
            self._level = level
            self._level_rngs = [rngs[z["tree"]] for z in nodes]
            t0 = time.perf_counter()
            lv_rows = int(sum(max(0, z["end"] - z["start"]) for z in nodes if z["built"]))
            self.hist_rows_total += lv_rows
            with trace_range(f"gbdt.level{level}.hist_split"):
                hist = self._build_and_split(nodes, n_built, gg, w, pos2row, hist_prev)
                best = hist["best"]            # per slot: (feat, bin, gain, lw, ls, rw, rs, valid)
            self.timings["split"] += time.perf_counter() - t0
            lv_stat = {"level": level, "nodes": len(nodes), "built": int(n_built), "hist_rows": lv_rows,
                       "hist_split_ms": (time.perf_counter() - t0) * 1e3}
            level_log.append(lv_stat)
            # decisions ------------------------------------------------------------------
            split_feat = np.full(len(nodes), -1, dtype=np.int32)
            split_bin = np.full(len(nodes), -1, dtype=np.int32)
            cat_left = np.zeros((len(nodes), 8), dtype=np.uint32)
            children = []
            last = level + 1 >= c.max_depth
            allowed = None
            if c.max_leaves > 0:
                # MaxLeaves (DTMaster :543-605, 1063-1071): split the candidates with the highest
                # wgtCnt-ratio x gain first while each tree's leaf budget lasts
                allowed = set()
                for t in range(T):
                    cands = sorted((-(float(best[z["slot"]][2]) * float(trees[t].wgt_cnt[z["id"]])), z["slot"])
                                   for z in nodes if z["tree"] == t and best[z["slot"]][7])
                    room = max(0, c.max_leaves - n_leaves[t])
                    if c.max_batch_split > 0:   # DTMaster :360 intends this cap (its loop never counts)
                        room = min(room, c.max_batch_split)
                    allowed |= {s_ for _, s_ in cands[:room]}
            for z in nodes:
                s_ = z["slot"]
                f, b, gain, lw, ls, rw, rs, ok = best[s_]
                nid = z["id"]
                if not ok or (allowed is not None and s_ not in allowed):
                    continue
                tree = trees[z["tree"]]
                n_leaves[z["tree"]] += 1
                f = int(f)
                tree.feat[nid] = f
                tree.gain[nid] = gain
                tree.features_used.append(f)
                if d.is_cat[f]:
                    order = hist["cat_order"][s_][f]
                    left_bins = order[: int(b) + 1]
                    for lb in left_bins:       # (int: a uint8 shift stays uint8 under NumPy 2)
                        lb = int(lb)
                        cat_left[s_, lb >> 5] |= np.uint32(1 << (lb & 31))
                    tree.cat_left[nid] = cat_left[s_]
                    tree.thr[nid] = -1
                else:
                    tree.thr[nid] = int(b)
                    split_bin[s_] = int(b)
                split_feat[s_] = f
                for cid, cw, cs in ((2 * nid, lw, ls), (2 * nid + 1, rw, rs)):
                    tree.exists[cid] = True
                    tree.value[cid] = cs / cw if cw != 0 else 0.0
                    tree.wgt_cnt[cid] = cw
                if "class_lr" in hist:
                    tree.class_value[2 * nid], tree.class_value[2 * nid + 1] = hist["class_lr"][s_]
                children.append((z, lw, rw))
            fuse = self._fuse if (self.gpu and T == 1) else None
            if fuse is not None:
                tree0 = trees[0]
                nv = np.zeros((3, len(nodes)), dtype=np.float32)
                for z in nodes:
                    nv[0, z["slot"]] = tree0.value[z["id"]]
                    if split_feat[z["slot"]] >= 0:
                        nv[1, z["slot"]] = tree0.value[2 * z["id"]]
                        nv[2, z["slot"]] = tree0.value[2 * z["id"] + 1]
                leaf_vals = _h2d(nv, self.dev)
            if last or not children:
                if fuse is not None:     # every remaining row gets its final leaf (child) value
                    self._leaf_update(nodes, split_feat, split_bin, cat_left, pos2row, pos_node, leaf_vals, fuse)
                break
            # next level's nodes: build the globally smaller child, derive the other (identical on
            # all ranks); their slots are fixed now so the partition scatter writes final slot ids
            new_nodes = []
            for z, lw, rw in children:
                left_built = lw <= rw
                new_nodes.append({"tree": z["tree"], "id": 2 * z["id"], "built": left_built, "parent": z["slot"]})
                new_nodes.append({"tree": z["tree"], "id": 2 * z["id"] + 1, "built": not left_built,
                                  "parent": z["slot"]})
            for s_, nz in enumerate(sorted(new_nodes, key=_slot_key)):
                nz["slot"] = s_
            child_slots = {new_nodes[2 * i]["parent"]: (new_nodes[2 * i]["slot"], new_nodes[2 * i + 1]["slot"])
                           for i in range(len(children))}
            # partition rows of split nodes -----------------------------------------------
            t0 = time.perf_counter()
            with trace_range(f"gbdt.level{level}.partition"):
                pos2row, pos_node, ranges = self._partition(nodes, split_feat, split_bin, cat_left, pos2row,
                                                            pos_node, child_slots,
                                                            (leaf_vals, fuse) if fuse is not None else None)
            self.timings["partition"] += time.perf_counter() - t0
            lv_stat["partition_ms"] = (time.perf_counter() - t0) * 1e3
            for i, nz in enumerate(new_nodes):
                lo, mid, hi = ranges[nz["parent"]]
                nz["start"], nz["end"] = (lo, mid) if i % 2 == 0 else (mid, hi)
            hist_prev = hist["hist"]
            nodes = new_nodes
        self._nmod, self._npos = 0, n
        return trees

    # ------------------------------------------------------------------------------------
    def _pipelined(self, T: int) -> bool:
        """Device decisions + device node ranges for this growth (see _grow_levels_dev)."""
        c = self.cfg
        return (DEV_DECIDE and self.gpu and not c.is_multiclass and c.max_leaves <= 0
                and T * 2 ** max(0, c.max_depth - 2) <= 512)

    def _grow_levels_dev(self, trees, rngs, nodes, pos2row, pos_node, w, gg, level_log, n_leaves):
        """The level loop with one host sync per level, hidden behind the partition.

        Per level the GPU runs, back to back: histogram items resolved to row ranges on the device
        (shifu_gbdt_items_fix), the histograms, the split scan, the decisions (shifu_gbdt_decide:
        best feature per node, split bin / categorical set, leaf values, the children's next-level
        slots), the partition (flags, per-node counts + the children's row ranges, scatter) -- or
        on the last level the fused leaf update.  The host waits only for the decisions' copy,
        then mirrors them into the Tree objects and builds the next level's items while the
        partition runs.  Items are sized from estimated child sizes (parent rows x child weight
        share) because the exact counts are still on the GPU; the chunking only balances work,
        the integer histograms do not depend on it.  The exact counts arrive one level later
        (pinned copy behind the scatter) for the row statistics.  Same trees as the host path
        (tests/test_gbdt.py: pipelined vs SHIFU_GBDT_DEV_DECIDE=0)."""
        from ..ops import _native as nat
        c, d, dev = self.cfg, self.data, self.dev
        st = nat.stream_of(d.y)
        fuse = self._fuse if len(trees) == 1 else None
        cat_any = bool(d.is_cat.any())
        nodes.sort(key=_slot_key)
        for s_, z in enumerate(nodes):
            z["slot"] = s_
        if RANGE_NODES:          # positions find their node from the sorted node ranges
            pos_node = None
        rng = _h2d(np.array([[z["start"] for z in nodes], [z["end"] for z in nodes]], np.int32), dev)
        nval = _h2d(np.array([trees[z["tree"]].value[z["id"]] for z in nodes], np.float32), dev)
        hist_prev = None
        nleft_prev = None            # pinned per-node left counts of the previous partition
        for level in range(1, c.max_depth):
            nn = len(nodes)
            last = level + 1 >= c.max_depth
            slot_of = {(z["tree"], z["id"]): z["slot"] for z in nodes}
            for z in nodes:
                if not z["built"]:
                    z["sib_slot"] = slot_of[(z["tree"], z["id"] ^ 1)]
            n_built = sum(1 for z in nodes if z["built"])
            self._root_level = level == 1
            self._level = level
            self._level_rngs = [rngs[z["tree"]] for z in nodes]
            t0 = time.perf_counter()
            with trace_range(f"gbdt.level{level}.hist_split"):
                h = self._build_and_split(nodes, n_built, gg, w, pos2row, hist_prev,
                                          rng=rng if level > 1 else None, raw=True)
                meta = _h2d(np.array([[z["tree"] for z in nodes], [z["id"] for z in nodes],
                                      [int(z["built"]) for z in nodes]], np.int32), dev)
                i32 = dict(dtype=torch.int32, device=dev)
                sf, sb, chl, chr_ = (torch.empty(nn, **i32) for _ in range(4))
                cl = torch.empty(nn, 8, **i32)
                lv = torch.empty(3, nn, dtype=torch.float32, device=dev)
                nxt = torch.empty(max(1, 2 * nn), dtype=torch.float32, device=dev)
                best_d = torch.empty(nn, 8, dtype=torch.float32, device=dev)
                nat.call_hip("shifu_gbdt_decide", h["cand"], self.F, nn, meta, nval, h["cat_order"], self.is_cat_t,
                             int(last), best_d, sf, sb, cl, chl, chr_, lv, nxt, st)
                best_h = torch.empty(nn, 8, dtype=torch.float32, pin_memory=True)
                best_h.copy_(best_d, non_blocking=True)
                cl_h = None
                if cat_any:
                    cl_h = torch.empty(nn, 8, dtype=torch.int32, pin_memory=True)
                    cl_h.copy_(cl, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            self.timings["split"] += time.perf_counter() - t0
            t1 = time.perf_counter()
            part = None
            with trace_range(f"gbdt.level{level}.partition"):
                if not last:
                    part = self._partition_dev(nn, rng, sf, sb, cl, chl, chr_, lv, pos2row, pos_node, fuse)
                elif fuse is not None:
                    self._leaf_update_dev(nn, rng, sf, sb, cl, lv, pos2row, pos_node, fuse)
            self.timings["partition"] += time.perf_counter() - t1
            ev.synchronize()
            # exact ranges of this level's nodes (the previous partition's counts came before ev)
            if nleft_prev is not None:
                nl = nleft_prev.numpy()
                for z in nodes:
                    lo, hi = z["prange"]
                    k = int(nl[z["parent"]])
                    z["start"], z["end"] = (lo, lo + k) if z["id"] % 2 == 0 else (lo + k, hi)
                    z.pop("m", None)
            lv_rows = int(sum(_zm(z) for z in nodes if z["built"]))
            self.hist_rows_total += lv_rows
            level_log.append({"level": level, "nodes": nn, "built": int(n_built), "hist_rows": lv_rows,
                              "hist_split_ms": (time.perf_counter() - t0) * 1e3})
            # the host mirror of the device decisions
            b = best_h.numpy().astype(np.float64)
            clh = cl_h.numpy().view(np.uint32) if cl_h is not None else None
            if DECIDE_CHECK:
                self._check_decisions(h, nodes, b, clh, sf, sb, chl, chr_, last)
            children = []
            for z in nodes:
                s_ = z["slot"]
                f, bn, gain, lw, ls, rw, rs, ok = b[s_]
                if not ok:
                    continue
                tree = trees[z["tree"]]
                nid = z["id"]
                n_leaves[z["tree"]] += 1
                f = int(f)
                tree.feat[nid] = f
                tree.gain[nid] = gain
                tree.features_used.append(f)
                if d.is_cat[f]:
                    tree.cat_left[nid] = clh[s_].copy()
                    tree.thr[nid] = -1
                else:
                    tree.thr[nid] = int(bn)
                for cid, cw, cs in ((2 * nid, lw, ls), (2 * nid + 1, rw, rs)):
                    tree.exists[cid] = True
                    tree.value[cid] = cs / cw if cw != 0 else 0.0
                    tree.wgt_cnt[cid] = cw
                children.append((z, lw, rw))
            if last or not children:
                # fused: the leaf update (last level) or the partition's flag pass (no split: every
                # row got its node's value) already moved pred
                if fuse is not None:
                    self._leaf_done = True
                break
            new_nodes = []
            for z, lw, rw in children:
                pm, tot = _zm(z), lw + rw
                for side, cw in ((0, lw), (1, rw)):
                    built = (lw <= rw) if side == 0 else not (lw <= rw)
                    est = (int(round(pm * cw / tot)) if tot > 0 else pm // 2)
                    if cw > 0:
                        est = max(1, est)
                    new_nodes.append({"tree": z["tree"], "id": 2 * z["id"] + side, "built": built,
                                      "parent": z["slot"], "prange": (z["start"], z["end"]), "m": min(est, pm)})
            new_nodes.sort(key=_slot_key)
            for s_, nz in enumerate(new_nodes):
                nz["slot"] = s_
            pos2row, pos_node, rng, nleft_prev = part
            nval = nxt
            hist_prev = h["hist"]
            nodes = new_nodes

    def _check_decisions(self, h, nodes, b, clh, sf, sb, chl, chr_, last):
        """SHIFU_GBDT_DECIDE_CHECK=1: the device decisions against _select_best + the host's
        categorical sets and slot order on the same candidates (debug; syncs)."""
        nn = len(nodes)
        ref = self._select_best(h["cand"], nn)
        co = None if h["cat_order"] is None else h["cat_order"].cpu().numpy()
        sf_d, sb_d = sf.cpu().numpy(), sb.cpu().numpy()
        chl_d, chr_d = chl.cpu().numpy(), chr_.cpu().numpy()
        kids = []
        for z in nodes:
            s_ = z["slot"]
            f, bn, gain, lw, ls, rw, rs, ok = ref[s_]
            got = tuple(float(v) for v in b[s_])
            want = (float(f), float(bn), gain, lw, ls, rw, rs, float(ok))
            if ok and got != want:
                raise AssertionError(f"decide: slot {s_} best {got} != host {want}")
            if bool(got[7]) != ok:
                raise AssertionError(f"decide: slot {s_} ok {got[7]} != host {ok}")
            exp_sf = f if ok else -1
            exp_sb = int(bn) if ok and not self.data.is_cat[f] else -1
            if sf_d[s_] != exp_sf or sb_d[s_] != exp_sb:
                raise AssertionError(f"decide: slot {s_} split ({sf_d[s_]}, {sb_d[s_]}) != host ({exp_sf}, {exp_sb})")
            words = np.zeros(8, np.uint32)
            if ok and self.data.is_cat[f]:
                for lb in co[s_][f][: int(bn) + 1]:
                    words[lb >> 5] |= np.uint32(1 << (int(lb) & 31))
            if clh is not None and not np.array_equal(words, clh[s_]):
                raise AssertionError(f"decide: slot {s_} cat set {clh[s_].tolist()} != host {words.tolist()} "
                                     f"(f {f} bin {bn} order {co[s_][f][:int(bn) + 1].tolist()})")
            if ok and not last:
                for side, built in ((0, lw <= rw), (1, not lw <= rw)):
                    kids.append(((not built, z["tree"], 2 * z["id"] + side), s_, side))
        kids.sort()
        for slot, (_, s_, side) in enumerate(kids):
            got = chl_d[s_] if side == 0 else chr_d[s_]
            if got != slot:
                raise AssertionError(f"decide: slot {s_} side {side} child slot {got} != host {slot}")

    def _partition_dev(self, nn, rng, sf, sb, cl, chl, chr_, lv, pos2row, pos_node, fuse):
        """The partition with every per-node input on the device (decide kernel outputs, node
        ranges): flags, per-node counts + the children's ranges, scatter.  Returns the new
        position arrays, the next level's ranges [2, 2 nn] and a pinned copy of the left counts."""
        from ..ops import _native as nat
        d = self.data
        st = nat.stream_of(d.y)
        n = self._npos
        nw = (n + 63) // 64
        fbits = torch.empty(nw, dtype=torch.int64, device=self.dev)
        wcnt = torch.empty(nw, dtype=torch.int32, device=self.dev)
        pred, scale = fuse if fuse is not None else (None, 0.0)
        rb = self._root_bins()
        ri = self._range_index(nn, rng) if pos_node is None else (None, None, None, 0)
        nat.call_hip("shifu_gbdt_partition_flag", d.kbins, d.group_stride, rb,
                     self._root_stride() if rb is not None else 0, pos2row, pos_node, sf, sb, cl, self.is_cat_t,
                     fbits, wcnt, n, self._nmod, pred, lv[0] if pred is not None else None, None, None,
                     float(scale), 0, *ri, st)
        wpre = torch.cumsum(wcnt, 0, dtype=torch.int32) - wcnt
        cbn = torch.empty(2, nn, dtype=torch.int32, device=self.dev)
        new_rng = torch.empty(2, 2 * nn, dtype=torch.int32, device=self.dev)
        nat.call_hip("shifu_gbdt_node_counts", fbits, wpre, rng[0], rng[1], nn, cbn[0], cbn[1], chl, chr_,
                     new_rng[0], new_rng[1], st)
        new_p2r = torch.empty_like(pos2row)
        new_pn = torch.empty_like(pos_node) if pos_node is not None else None
        wg = self._wg_pos
        nw_, ng_ = (torch.empty_like(wg[0]), torch.empty_like(wg[1])) if wg is not None else (None, None)
        nat.call_hip("shifu_gbdt_partition_scatter", pos2row, pos_node, fbits, wpre, rng[0], cbn[1], cbn[0],
                     sf, chl, chr_, new_p2r, new_pn, None if wg is None else wg[0],
                     None if wg is None else wg[1], nw_, ng_, n, *ri, st)
        if wg is not None:
            self._wg_pos = (nw_, ng_)
        nleft = torch.empty(nn, dtype=torch.int32, pin_memory=True)
        nleft.copy_(cbn[1], non_blocking=True)
        return new_p2r, new_pn, new_rng, nleft

    def _leaf_update_dev(self, nn, rng, sf, sb, cl, lv, pos2row, pos_node, fuse):
        """_leaf_update with the decisions and node ranges on the device."""
        from ..ops import _native as nat
        d = self.data
        pred, scale = fuse
        rb = self._root_bins()
        st = nat.stream_of(d.y)
        if LEAF_WINDOW and self._nmod == 0 and nn <= 1024:
            nw = ((d.n + LEAF_W - 1) // LEAF_W + 7) // 8 * 8
            bounds = torch.empty(nn * (nw + 1), dtype=torch.int32, device=self.dev)
            nat.call_hip("shifu_gbdt_leaf_window", d.kbins, d.group_stride, rb,
                         self._root_stride() if rb is not None else 0, pos2row, rng[0], rng[1], nn, d.n, LEAF_W,
                         LEAF_Y, bounds, sf, sb, cl, self.is_cat_t, pred, lv[0], lv[1], lv[2], float(scale), st)
            return
        ri = self._range_index(nn, rng) if pos_node is None else (None, None, None, 0)
        nat.call_hip("shifu_gbdt_partition_flag", d.kbins, d.group_stride, rb,
                     self._root_stride() if rb is not None else 0, pos2row, pos_node, sf, sb, cl, self.is_cat_t,
                     None, None, self._npos, self._nmod, pred, lv[0], lv[1], lv[2], float(scale), 1, *ri, st)

    def _range_index(self, nn, rng):
        """The level's node ranges sorted by start (range_node in gbdt_kernels.hip): the partition
        finds a position's node from these instead of a per-position node array."""
        from ..ops import _native as nat
        r_start = torch.empty(nn, dtype=torch.int32, device=self.dev)
        r_slot = torch.empty(nn, dtype=torch.int32, device=self.dev)
        nat.call_hip("shifu_gbdt_range_index", rng[0], rng[1], nn, r_start, r_slot, nat.stream_of(self.data.y))
        return r_start, r_slot, rng[1], nn

    # ------------------------------------------------------------------------------------
    def _make_items(self, nodes, n_built, est=False, align=1):
        """Work items [n, 4] = (node_slot, lo, hi, group) for the built nodes, chunked for
        parallelism, and node_items [n_nodes, n_groups, max_items] (item ids, -1 padded).
        Vectorized over all nodes at once (it runs on the host between two GPU launches of every
        level); order: node, quad, chunk, sub-group.  ``est``: the node sizes z["m"] are estimates
        and the row ranges live on the device -- items hold (slot, chunk, n_chunks, group) and
        shifu_gbdt_items_fix turns them into row ranges before the histogram launch."""
        G = self.ngroups
        Q = (G + 3) // 4
        bz = [z for z in nodes if z["built"] and _zm(z) > 0]
        if not bz:
            return np.zeros((0, 4), np.int32), np.full((len(nodes), G, 1), -1, np.int32), 1
        slot = np.array([z["slot"] for z in bz], np.int64)
        start = np.zeros(len(bz), np.int64) if est else np.array([z["start"] for z in bz], np.int64)
        m = np.array([_zm(z) for z in bz], np.int64)
        rows_built = sum(_zm(z) for z in nodes if z["built"])
        if self.items_per_node_group is None:
            # below the root, levels with few built nodes run fewer, longer items (less per-item LDS
            # zeroing and slab traffic; levels 3 / 4 of the balanced bench 13.1 / 12.3 vs 13.9 /
            # 12.5 ms, levels with 8+ nodes lose with it: profiles/r6/gbdt/items_per_level_r6.txt)
            target = TARGET_ITEMS_FEW if (not getattr(self, "_root_level", True) and n_built <= 4) else TARGET_ITEMS
            k = np.maximum(1, np.rint(target * (m / max(1, rows_built)) / G).astype(np.int64))
            k = np.minimum(np.minimum(k, np.maximum(1, m // 4096)), 64)
        else:
            k = np.full(len(bz), int(self.items_per_node_group), np.int64)
        step = (m + k - 1) // k
        if align > 1:       # chunk boundaries on whole row tiles (the tiled root pass skips its row mask)
            step = (step + align - 1) // align * align
        k = (m + step - 1) // step                          # chunks that are non-empty
        # one row per (node, quad, chunk, sub-group): the 4 groups of one 128-B record and row
        # range are consecutive items (one XCD, gbdt_kernels.hip xcd_remap) and share its lines
        per = Q * k * 4
        tot = int(per.sum())
        nd = np.repeat(np.arange(len(bz)), per)
        r = np.arange(tot) - np.repeat(np.cumsum(per) - per, per)      # index inside the node's block
        kk = k[nd]
        q, rem = r // (kk * 4), r % (kk * 4)
        ch, sg = rem // 4, rem % 4
        grp = q * 4 + sg
        if est:
            lo, hi = ch, kk
        else:
            lo = start[nd] + ch * step[nd]
            hi = np.minimum(start[nd] + m[nd], lo + step[nd])
        keep = grp < G
        items = np.stack([slot[nd], lo, hi, grp], 1)[keep].astype(np.int32)
        max_items = int(k.max())
        ni = np.full((len(nodes), G, max_items), -1, dtype=np.int32)
        ni[slot[nd][keep], grp[keep], ch[keep]] = np.arange(len(items), dtype=np.int32)
        return items, ni, max_items

    def _hist_allreduce(self, h: torch.Tensor) -> None:
        """All-reduce one level's built-node histograms (one bucket per level), timed: HIP events
        on the GPU (read when the tree is done), host wall time on the CPU (gloo is synchronous)."""
        if dist.info().world_size <= 1:
            return
        with trace_range("gbdt.hist_allreduce"):
            if h.is_cuda:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                dist.all_reduce_(h)
                e1.record()
                self._ar_events.append((e0, e1))
            else:
                t0 = time.perf_counter()
                dist.all_reduce_(h)
                self._ar_events.append((time.perf_counter() - t0) * 1e3)

    def _allreduce_ms(self) -> float:
        """Histogram all-reduce time since the last call (synchronises on pending events)."""
        ms = 0.0
        for e in self._ar_events:
            if isinstance(e, tuple):
                e[1].synchronize()
                ms += e[0].elapsed_time(e[1])
            else:
                ms += e
        self._ar_events = []
        return ms

    def _build_and_split(self, nodes, n_built, g, w, pos2row, hist_prev, rng=None, raw=False):
        """raw (GPU): return the split candidates [nn, F, 8] and the categorical orders on the
        device (the decisions are made by shifu_gbdt_decide); rng: the level's node row ranges
        [2, nn] on the device (histogram items sized from estimates)."""
        F = self.F
        nn = len(nodes)
        mask = self._node_feature_mask(nn)
        if self.cfg.is_multiclass:
            return self._build_and_split_multi(nodes, n_built, g, w, pos2row, hist_prev, mask)
        imp = IMPURITY_IDS[self.cfg.impurity]
        min_inst = float(self.cfg.min_instances_per_node)
        min_gain = float(self.cfg.min_info_gain)
        # GPU: the split kernel writes every (node, feature, bin) entry (built: mode 0, derived: mode 1),
        # so no zero fill of the level's histograms (up to 64 nodes x 4 MB)
        alloc = torch.empty if self.gpu else torch.zeros
        hist = alloc(nn, 2, F, NB, dtype=torch.int64, device=self.dev)
        if self.gpu and raw:
            cand, cat_order = self._build_and_split_hip(nodes, n_built, g, w, pos2row, hist_prev, hist, mask,
                                                        imp, min_inst, min_gain, rng=rng, raw=True)
            return {"hist": hist, "cand": cand, "cat_order": cat_order}
        if self.gpu:
            best, cat_order = self._build_and_split_hip(nodes, n_built, g, w, pos2row, hist_prev, hist, mask,
                                                        imp, min_inst, min_gain)
        else:
            best, cat_order = self._build_and_split_torch(nodes, n_built, g, w, pos2row, hist_prev, hist, mask,
                                                          imp, min_inst, min_gain)
        return {"hist": hist, "best": best, "cat_order": cat_order}

    def _select_best(self, cand: torch.Tensor, nn: int):
        """cand [nn, F, 8] -> per node best (lowest feature on ties)."""
        gains = cand[:, :, 0].clone()
        valid = cand[:, :, 6] > 0
        gains[~valid] = -float("inf")
        fbest = torch.argmax(gains, dim=1)                       # first max -> lowest feature
        rows = cand[torch.arange(nn, device=cand.device), fbest]  # [nn, 8]
        out = torch.cat([fbest.unsqueeze(1).float(), rows[:, 1:2], rows[:, 0:1], rows[:, 2:6], rows[:, 6:7]], 1)
        out = torch.cat([out, valid.any(dim=1, keepdim=True).float()], 1).cpu().double().numpy()   # one sync
        ok = out[:, -1] > 0
        res = []
        for i in range(nn):
            f, b, gain, lw, ls, rw, rs, v = out[i, :8]
            res.append((int(f), int(b), float(gain), float(lw), float(ls), float(rw), float(rs), bool(ok[i])))
        return res

    def _build_and_split_hip(self, nodes, n_built, g, w, pos2row, hist_prev, hist, mask, imp, min_inst, min_gain,
                             rng=None, raw=False):
        from ..ops import _native as nat
        d = self.data
        F, nn = self.F, len(nodes)
        st = nat.stream_of(d.y)
        tiled_root = self._root_level and self._nmod == 0 and ROOT_U32 and self._root_bins() is not None
        items, ni, max_items = self._make_items(nodes, n_built, est=rng is not None, align=128 if tiled_root else 1)
        ni_t = _h2d(ni, self.dev)
        feat_list = torch.arange(F, dtype=torch.int32, device=self.dev)
        cand = torch.zeros(nn, F, 8, dtype=torch.float32, device=self.dev)
        cat_order = torch.zeros(nn, F, NB, dtype=torch.uint8, device=self.dev) if d.is_cat.any() else None
        t0 = time.perf_counter()
        if len(items):
            it = _h2d(items, self.dev)
            if rng is not None:
                nat.call_hip("shifu_gbdt_items_fix", it, len(items), rng[0], rng[1], st)
            ls = self.level_stats
            if ls is not None:          # per-level histogram roofline (bench --gbdt-levels)
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            if self._root_level and self._nmod == 0 and ROOT_U32:
                slab = self._root_slab(items, it, w, g, st)
            else:
                slab = torch.empty(len(items), 2, FG, NB, dtype=torch.int64, device=self.dev)
                p2r = None if self._root_level else pos2row      # root: positions are rows
                by_pos = p2r is not None and self._wg_pos is not None
                wv, gv = self._wg_pos if by_pos else (w, g)
                rows_built = sum(_zm(z) for z in nodes if z["built"])
                if HIST64 and not self._root_level and rows_built >= HIST64_MIN_NODE_ROWS * max(1, n_built):
                    pairs = _group_pairs(items)     # half-record blocks: groups 2j, 2j + 1 paired
                    pairs_t = _h2d(pairs, self.dev)        # lives until the level's D2H below
                    nat.call_hip("shifu_gbdt_hist64", d.kbins, d.group_stride, p2r, wv, gv, int(by_pos), it,
                                 len(items), pairs_t, len(pairs), slab, F, self.scale_w, self.scale_g,
                                 self._nmod, st)
                else:
                    nat.call_hip("shifu_gbdt_hist", d.kbins, d.group_stride, QF, p2r, wv, gv, int(by_pos), it,
                                 len(items), slab, F, self.scale_w, self.scale_g, self._nmod, 0, st)
            if ls is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                rows = int(sum(_zm(z) for z in nodes if z["built"]))
                ls.append({"level": self._level, "nodes_built": int(n_built), "rows": rows, "ev": (ev0, ev1)})
        else:
            slab = torch.zeros(1, 2, FG, NB, dtype=torch.int64, device=self.dev)
        built = _h2d(np.asarray([z["slot"] for z in nodes if z["built"]], np.int32), self.dev)
        derived = [z for z in nodes if not z["built"]]
        if n_built:
            nat.call_hip("shifu_gbdt_split", slab.data_ptr(), ni_t.data_ptr(), max_items, None, None, None,
                         hist.data_ptr(), built.data_ptr(), n_built, feat_list.data_ptr(), F,
                         self.nbins_t.data_ptr(), self.is_cat_t.data_ptr(), None, cand.data_ptr(), None, F, 0, imp,
                         0, min_inst, min_gain, 1.0 / self.scale_w, 1.0 / self.scale_g, st)
        self.timings["hist"] += time.perf_counter() - t0
        # cross-rank reduction of the built-node histograms (one RCCL bucket per level)
        if n_built:
            self._hist_allreduce(hist[:n_built])
        mptr = None if mask is None else mask.data_ptr()
        cptr = None if cat_order is None else cat_order.data_ptr()
        if n_built:
            nat.call_hip("shifu_gbdt_split", slab.data_ptr(), ni_t.data_ptr(), max_items, None, None, None,
                         hist.data_ptr(), built.data_ptr(), n_built, feat_list.data_ptr(), F,
                         self.nbins_t.data_ptr(), self.is_cat_t.data_ptr(), mptr, cand.data_ptr(), cptr, F, 2, imp,
                         1, min_inst, min_gain, 1.0 / self.scale_w, 1.0 / self.scale_g, st)
        if derived:
            dl = _h2d(np.asarray([z["slot"] for z in derived], np.int32), self.dev)
            par = np.zeros(nn, np.int32)
            sib = np.zeros(nn, np.int32)
            for z in derived:
                par[z["slot"]] = z["parent"]
                sib[z["slot"]] = z["sib_slot"]
            par_t = _h2d(par, self.dev)
            sib_t = _h2d(sib, self.dev)
            nat.call_hip("shifu_gbdt_split", slab.data_ptr(), ni_t.data_ptr(), max_items, hist_prev.data_ptr(),
                         par_t.data_ptr(), sib_t.data_ptr(), hist.data_ptr(), dl.data_ptr(), len(derived),
                         feat_list.data_ptr(), F, self.nbins_t.data_ptr(), self.is_cat_t.data_ptr(), mptr,
                         cand.data_ptr(), cptr, F, 1, imp, 1, min_inst, min_gain, 1.0 / self.scale_w,
                         1.0 / self.scale_g, st)
        if raw:
            return cand, cat_order
        best = self._select_best(cand, nn)
        co = None if cat_order is None else cat_order.cpu().numpy()
        return best, co

    def _root_bins(self):
        """A feature-tiled copy of the (quad-blocked) bins, [G][NT][32][128] with NT = ceil(N/128),
        made once when HBM has room for it (SHIFU_GBDT_ROOT_G32=0: never).  The dense root pass
        streams whole 4-KiB tiles (gbdt_root_tile_kernel), and the partition passes read a row's
        split-feature byte from a 128-B line of 128 consecutive rows of that feature, shared by the
        node's other rows in the window (the quad records made every row fetch its own line).
        None: use the quad records."""
        d = self.data
        if not ROOT_G32 or d.bins_dptr is not None or d.bins.device.type != "cuda":
            return None
        c = getattr(self, "_g32", None)
        if c is None:
            G, n = self.ngroups, d.n
            nt = (n + 127) // 128
            need = G * nt * 4096
            from ..utils.device import free_hbm
            free = free_hbm(self.dev)
            if free < need * 1.1 + (6 << 30):
                _log.info("GBDT root: no room for the feature-tiled bins copy (%.1f GB); quad records", need / 1e9)
                self._g32 = False
                return None
            from ..ops import _native as nat
            b = torch.empty(G, nt * 4096, dtype=torch.uint8, device=self.dev)
            nat.call_hip("shifu_gbdt_tile_bins", d.kbins, d.group_stride, n, G, b, nt * 4096, nat.stream_of(d.y))
            self._g32 = c = b
        return c if c is not False else None

    def _root_stride(self) -> int:
        """Group stride (bytes) of the feature-tiled root copy."""
        return (self.data.n + 127) // 128 * 4096

    def _root_slab(self, items, it, w, g, st):
        """Root-level slabs from the two u32 histogram modes: sum w (mode 1) is built once and
        kept while the weight tensor is the same unmodified object (no bagging sub-sample, the
        usual GBT case), sum w*g (mode 2) is rebuilt every tree.  One u32 LDS atomic per (row,
        feature) instead of the packed u64: about half the root level's histogram time."""
        from ..ops import _native as nat
        d = self.data
        key = (w._version, self.scale_w, hash(items.tobytes()), d.bins.data_ptr(), d.bins_dptr)
        c = getattr(self, "_root_cache", None)
        rb = self._root_bins()
        q = None
        if rb is not None:
            q = getattr(self, "_root_q", None)
            if q is None or q.numel() < self._root_stride() // 32:
                q = self._root_q = torch.empty(self._root_stride() // 32, dtype=torch.int32, device=self.dev)
        if c is None or c[0] is not w or c[1] != key:
            slab = torch.empty(len(items), 2, FG, NB, dtype=torch.int64, device=self.dev)
            if rb is not None:
                nat.call_hip("shifu_gbdt_hist_root_tile", rb, self._root_stride(), d.n, w, g, it, len(items), slab,
                             self.scale_w, self.scale_g, 1, q, st)
            else:
                nat.call_hip("shifu_gbdt_hist", d.kbins, d.group_stride, QF, None, w, g, 0,
                             it, len(items), slab, self.F, self.scale_w, self.scale_g, 0, 1, st)
            self._root_cache = (w, key, slab)          # holds w: its storage cannot be re-issued
        slab = self._root_cache[2]
        if rb is not None:           # dense root pass over the feature tiles (every line fully used)
            nat.call_hip("shifu_gbdt_hist_root_tile", rb, self._root_stride(), d.n, w, g, it, len(items), slab,
                         self.scale_w, self.scale_g, 2, q, st)
        elif ROOT_QUAD:
            # sum w*g over whole 128-B records: one block per (row range, quad) consumes every
            # line it fetches (gbdt_kernels.hip gbdt_root_quad_kernel)
            first = np.nonzero(items[:, 3] % 4 == 0)[0]
            q = np.stack([first, items[first, 1], items[first, 2], items[first, 3] // 4], 1).astype(np.int32)
            qt = _h2d(np.ascontiguousarray(q), self.dev)
            nat.call_hip("shifu_gbdt_hist_root_quad", d.kbins, d.group_stride, w, g, qt, len(q), slab,
                         self.ngroups, self.scale_g, st)
        else:
            nat.call_hip("shifu_gbdt_hist", d.kbins, d.group_stride, QF, None, w, g, 0, it, len(items), slab, self.F,
                         self.scale_w, self.scale_g, 0, 2, st)
        return slab

    # ---- native multi-class RF (Entropy / Gini over C classes) ------------------------------
    def _class_hist(self, nodes, n_built, gc, w, pos2row, hist_prev, hist):
        """One class's (sum w, sum w*[y == c]) histograms of every node of the level: the packed
        HIP histogram kernel + slab reduction for the built nodes (all-reduced across ranks),
        parent - sibling for the derived ones."""
        d = self.data
        F = self.F
        if self.gpu:
            from ..ops import _native as nat
            st = nat.stream_of(d.y)
            items, ni, max_items = self._make_items(nodes, n_built)
            if n_built and len(items):
                ni_t = _h2d(ni, self.dev)
                it = _h2d(items, self.dev)
                slab = torch.empty(len(items), 2, FG, NB, dtype=torch.int64, device=self.dev)
                p2r = None if self._root_level else pos2row
                nat.call_hip("shifu_gbdt_hist", d.kbins, d.group_stride, QF, p2r, w, gc, 0, it, len(items), slab, F,
                             self.scale_w, self.scale_g, self._nmod, 0, st)
                built = _h2d(np.asarray([z["slot"] for z in nodes if z["built"]], np.int32), self.dev)
                feat_list = torch.arange(F, dtype=torch.int32, device=self.dev)
                cand = torch.zeros(len(nodes), F, 8, dtype=torch.float32, device=self.dev)
                nat.call_hip("shifu_gbdt_split", slab.data_ptr(), ni_t.data_ptr(), max_items, None, None, None,
                             hist.data_ptr(), built.data_ptr(), n_built, feat_list.data_ptr(), F,
                             self.nbins_t.data_ptr(), self.is_cat_t.data_ptr(), None, cand.data_ptr(), None, F, 0,
                             IMPURITY_IDS["variance"], 0, 0.0, 0.0, 1.0 / self.scale_w, 1.0 / self.scale_g, st)
            elif n_built:
                hist[:n_built].zero_()
        else:
            bins = self._codes().long()
            for z in nodes:
                if not z["built"]:
                    continue
                hist[z["slot"]].zero_()
                rows = pos2row[z["start"]: z["end"]].long()
                if rows.numel() == 0:
                    continue
                b = bins[rows % d.n]
                qw = torch.round(w[rows].double() * self.scale_w).long()
                qg = torch.round((w[rows] * gc[rows]).float().double() * self.scale_g).long()
                idx = (torch.arange(F).unsqueeze(0) * NB + b).reshape(-1)
                hist[z["slot"], 0].view(-1).index_add_(0, idx, qw.unsqueeze(1).expand(-1, F).reshape(-1))
                hist[z["slot"], 1].view(-1).index_add_(0, idx, qg.unsqueeze(1).expand(-1, F).reshape(-1))
        if n_built:
            self._hist_allreduce(hist[:n_built])
        for z in nodes:
            if not z["built"]:
                hist[z["slot"]] = hist_prev[z["parent"]] - hist[z["sib_slot"]]

    def _build_and_split_multi(self, nodes, n_built, g, w, pos2row, hist_prev, mask):
        """``Entropy`` / ``Gini`` split search over per-class bin statistics
        (Impurity.java:368-734): the class sums come from C runs of the packed histogram kernel
        (target = one-hot of the class), the gain scan is vectorized over (node, feature, bin)."""
        cfg, d = self.cfg, self.data
        C, F, nn = cfg.n_classes, self.F, len(nodes)
        yl = g.round().long()
        hists = []
        for c in range(C):
            gc = (yl == c).float().contiguous()
            h = torch.empty(nn, 2, F, NB, dtype=torch.int64, device=self.dev)
            self._class_hist(nodes, n_built, gc, w, pos2row, None if hist_prev is None else hist_prev[c], h)
            hists.append(h)
        H = torch.stack([h[:, 1] for h in hists], -1).double() * (1.0 / self.scale_g)     # [nn, F, NB, C]
        nb = self.nbins_t.long()
        binr = torch.arange(NB, device=self.dev)
        inb = binr[None, :] < nb[:, None]                                                 # [F, NB]
        cat_order = None
        if d.is_cat.any():
            # categorical bins ordered by the class-1 rate of (class 0 + class 1) (Entropy /
            # Gini getCategoricalOrderList); bins past the category count sort last
            den = H[..., 0] + H[..., 1]
            key = torch.where(den != 0, H[..., 1] / torch.where(den != 0, den, torch.ones_like(den)),
                              torch.zeros_like(den))
            key = torch.where(inb[None], key, torch.full_like(key, float("inf")))
            iscat = _h2d(d.is_cat.astype(bool), self.dev)
            key = torch.where(iscat[None, :, None], key, binr.double()[None, None, :].expand_as(key))
            order = torch.argsort(key, dim=2, stable=True)                                # [nn, F, NB]
            H = torch.gather(H, 2, order[..., None].expand(-1, -1, -1, C))
            cat_order = order.to(torch.uint8).cpu().numpy()
        L = torch.cumsum(H, 2)
        T = L[:, :, -1:, :]
        R = T - L
        lw, rw, tw = L.sum(-1), R.sum(-1), T.sum(-1)

        def impurity(X, s):
            p = X / torch.where(s > 0, s, torch.ones_like(s))[..., None]
            if cfg.impurity == "gini":
                return -(p * p).sum(-1)
            return -torch.where(p > 0, p * torch.log2(torch.where(p > 0, p, torch.ones_like(p))),
                                torch.zeros_like(p)).sum(-1)
        gain = impurity(T, tw) - torch.where(tw > 0, lw / tw, torch.zeros_like(lw)) * impurity(L, lw) \
            - torch.where(tw > 0, rw / tw, torch.zeros_like(rw)) * impurity(R, rw)
        ok = (binr[None, None, :] < (nb[None, :, None] - 1)) & (lw > cfg.min_instances_per_node) & \
            (rw > cfg.min_instances_per_node) & (gain > cfg.min_info_gain)
        if mask is not None:
            ok &= mask.bool()[:, :, None]
        g_m = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
        bbest = torch.argmax(g_m, dim=2)                                                  # first max bin
        gbest = torch.gather(g_m, 2, bbest[..., None])[..., 0]                            # [nn, F]
        fbest = torch.argmax(gbest, dim=1)                                                # lowest feature
        ar = torch.arange(nn, device=self.dev)
        b_sel = bbest[ar, fbest]
        g_sel = gbest[ar, fbest]
        Lc = L[ar, fbest, b_sel]                                                          # [nn, C]
        Rc = R[ar, fbest, b_sel]
        res = torch.stack([fbest.double(), b_sel.double(), g_sel, Lc.sum(-1), Lc[:, 1], Rc.sum(-1), Rc[:, 1],
                           torch.isfinite(g_sel).double(), Lc.argmax(-1).double(), Rc.argmax(-1).double()], 1)
        res = res.cpu().numpy()
        best, class_lr = [], []
        for i in range(nn):
            f, b, gn, lws, l1, rws, r1, v, cl, cr = res[i]
            best.append((int(f), int(b), float(gn) if v else 0.0, float(lws), float(l1), float(rws), float(r1),
                         bool(v)))
            class_lr.append((float(cl), float(cr)))
        return {"hist": hists, "best": best, "cat_order": cat_order, "class_lr": class_lr}

    def _build_and_split_torch(self, nodes, n_built, g, w, pos2row, hist_prev, hist, mask, imp, min_inst,
                               min_gain):
        """CPU oracle: same decomposition with torch ops (fp64 scan)."""
        d = self.data
        F, nn = self.F, len(nodes)
        bins = self._codes().long()
        for z in nodes:
            if not z["built"]:
                continue
            rows = pos2row[z["start"]: z["end"]].long()
            if rows.numel() == 0:
                continue
            b = bins[rows % d.n]                             # [m, F] (virtual rows of a forest batch)
            qw = torch.round(w[rows].double() * self.scale_w).long()
            if self._root_level and self._nmod == 0 and ROOT_U32:    # the u32 root mode's coarser grid
                qg = torch.round((w[rows] * g[rows]).float().double() * (self.scale_g / ROOT_G_DIV)).long() * ROOT_G_DIV
            else:
                qg = torch.round((w[rows] * g[rows]).float().double() * self.scale_g).long()
            idx = (torch.arange(F).unsqueeze(0) * NB + b).reshape(-1)
            hw = torch.zeros(F * NB, dtype=torch.int64)
            hg = torch.zeros(F * NB, dtype=torch.int64)
            hw.index_add_(0, idx, qw.unsqueeze(1).expand(-1, F).reshape(-1))
            hg.index_add_(0, idx, qg.unsqueeze(1).expand(-1, F).reshape(-1))
            hist[z["slot"], 0] = hw.view(F, NB)
            hist[z["slot"], 1] = hg.view(F, NB)
        if n_built:
            self._hist_allreduce(hist[:n_built])
        for z in nodes:
            if not z["built"]:
                hist[z["slot"]] = hist_prev[z["parent"]] - hist[z["sib_slot"]]
        cand = torch.zeros(nn, F, 8, dtype=torch.float32)
        cat_order = np.zeros((nn, F, NB), dtype=np.uint8) if d.is_cat.any() else None
        HW = hist[:, 0].double() * (1.0 / self.scale_w)
        HG = hist[:, 1].double() * (1.0 / self.scale_g)
        for s_ in range(nn):
            for f in range(F):
                if mask is not None and not mask[s_, f]:
                    continue
                cw = HW[s_, f].clone()
                cs = HG[s_, f].clone()
                nb = int(d.nbins[f])
                if d.is_cat[f]:
                    keys = [(1e300 if b >= nb else (float(cs[b] / cw[b]) if cw[b] != 0 else 4.9e-324), b)
                            for b in range(NB)]
                    order = [b for _, b in sorted(keys)]
                    cat_order[s_, f] = order
                    cw, cs = cw[order], cs[order]
                pw, ps = torch.cumsum(cw, 0), torch.cumsum(cs, 0)
                tw, ts = float(pw[-1]), float(ps[-1])
                best, bb = -1.0, -1
                for b in range(nb - 1):
                    lw, ls = float(pw[b]), float(ps[b])
                    rw, rs = tw - lw, ts - ls
                    if lw <= min_inst or rw <= min_inst:
                        continue
                    gain = _gain_py(imp, lw, ls, rw, rs)
                    if not gain > min_gain:
                        continue
                    if gain > best:
                        best, bb = gain, b
                if bb >= 0:
                    lw, ls = float(pw[bb]), float(ps[bb])
                    cand[s_, f] = torch.tensor([best, bb, lw, ls, tw - lw, ts - ls, 1.0, tw])
        return self._select_best(cand, nn), cat_order

    # ------------------------------------------------------------------------------------
    def _leaf_update(self, nodes, split_feat, split_bin, cat_left, pos2row, pos_node, leaf_vals, fuse):
        """Final level of a fused GBT tree: pred[row] += scale * value of the row's leaf (split nodes:
        the child its bin goes to).  Default: walked in row windows, each XCD updating its own
        windows' pred lines in its L2 (gbdt_leaf_window_kernel); SHIFU_GBDT_LEAF_WINDOW=0: the
        position-ordered partition-flag kernel without a flag output."""
        from ..ops import _native as nat
        d = self.data
        nn = len(nodes)
        pred, scale = fuse
        self._leaf_done = True
        rb = self._root_bins()
        st = nat.stream_of(d.y)
        if LEAF_WINDOW and self._nmod == 0 and nn <= 1024:
            starts = np.array([z["start"] for z in nodes], dtype=np.int32)
            ends = np.array([z["end"] for z in nodes], dtype=np.int32)
            meta = _h2d(np.concatenate([split_feat.astype(np.int32), split_bin.astype(np.int32),
                                        cat_left.view(np.int32).reshape(-1), starts, ends]), self.dev)
            sf, sb, cl = meta[:nn], meta[nn:2 * nn], meta[2 * nn:10 * nn]
            st_t, en_t = meta[10 * nn:11 * nn], meta[11 * nn:12 * nn]
            nw = ((d.n + LEAF_W - 1) // LEAF_W + 7) // 8 * 8
            bounds = torch.empty(nn * (nw + 1), dtype=torch.int32, device=self.dev)
            nat.call_hip("shifu_gbdt_leaf_window", d.kbins, d.group_stride, rb,
                         self._root_stride() if rb is not None else 0, pos2row, st_t, en_t, nn, d.n, LEAF_W, LEAF_Y,
                         bounds, sf, sb, cl, self.is_cat_t, pred, leaf_vals[0], leaf_vals[1], leaf_vals[2],
                         float(scale), st)
            return
        sf = _h2d(split_feat, self.dev)
        sb = _h2d(split_bin, self.dev)
        cl = _h2d(cat_left.view(np.int32), self.dev)
        nat.call_hip("shifu_gbdt_partition_flag", d.kbins, d.group_stride, rb, self._root_stride() if rb is not None else 0,
                     pos2row, pos_node, sf, sb, cl, self.is_cat_t, None, None, self._npos, self._nmod, pred, leaf_vals[0], leaf_vals[1], leaf_vals[2], float(scale),
                     1, None, None, None, 0, st)

    def _partition(self, nodes, split_feat, split_bin, cat_left, pos2row, pos_node, child_slots, leaf=None):
        d = self.data
        nn = len(nodes)
        n = self._npos                   # positions (T * N for a forest batch)
        starts = np.array([z["start"] for z in nodes], dtype=np.int64)
        ends = np.array([z["end"] for z in nodes], dtype=np.int64)
        # positions of unsplit nodes are never moved; mark non-split node positions -1
        if self.gpu:
            from ..ops import _native as nat
            st = nat.stream_of(d.y)
            child_l = np.full(nn, -1, np.int32)
            child_r = np.full(nn, -1, np.int32)
            for s_, (cl_, cr_) in child_slots.items():
                child_l[s_], child_r[s_] = cl_, cr_
            # every per-node array of the level in ONE upload: split feature / bin, categorical
            # left sets, node position ranges and child slots
            meta = _h2d(np.concatenate([split_feat.astype(np.int32), split_bin.astype(np.int32),
                                        cat_left.view(np.int32).reshape(-1), starts.astype(np.int32),
                                        ends.astype(np.int32), child_l, child_r]), self.dev)
            sf, sb = meta[:nn], meta[nn:2 * nn]
            cl = meta[2 * nn:10 * nn]
            st_t, en_t, chl_t, chr_t = (meta[(10 + k) * nn:(11 + k) * nn] for k in range(4))
            # left bits, one 64-bit word per 64 positions + the words' popcounts (exclusive-scanned):
            # the inclusive left count at p is wpre[p / 64] + popcount of the word's bits <= p
            nw = (n + 63) // 64
            fbits = torch.empty(nw, dtype=torch.int64, device=self.dev)
            wcnt = torch.empty(nw, dtype=torch.int32, device=self.dev)
            lv, (pred, scale) = leaf if leaf is not None else (None, (None, 0.0))
            # non-split nodes' rows get their leaf value here (fused GBT prediction update)
            rb = self._root_bins()        # feature-tiled copy when it exists
            nat.call_hip("shifu_gbdt_partition_flag", d.kbins, d.group_stride, rb, self._root_stride() if rb is not None else 0,
                         pos2row, pos_node, sf, sb, cl, self.is_cat_t, fbits, wcnt, n, self._nmod, pred, None if lv is None else lv[0], None, None,
                         float(scale), 0, None, None, None, 0, st)
            wpre = torch.cumsum(wcnt, 0, dtype=torch.int32) - wcnt
            # per node: left count before its start and #left, on the device; the scatter runs
            # before the host reads the counts (the D2H overlaps it)
            cbn = torch.empty(2, nn, dtype=torch.int32, device=self.dev)
            nat.call_hip("shifu_gbdt_node_counts", fbits, wpre, st_t, en_t, nn, cbn[0], cbn[1], None, None, None, None, st)
            new_p2r = torch.empty_like(pos2row)
            new_pn = torch.empty_like(pos_node)
            # tensors (not .data_ptr() of temporaries) so every buffer outlives the launch
            wg = self._wg_pos
            nw_, ng_ = (torch.empty_like(wg[0]), torch.empty_like(wg[1])) if wg is not None else (None, None)
            nat.call_hip("shifu_gbdt_partition_scatter", pos2row, pos_node, fbits, wpre, st_t, cbn[1], cbn[0],
                         sf, chl_t, chr_t, new_p2r, new_pn, None if wg is None else wg[0],
                         None if wg is None else wg[1], nw_, ng_, n, None, None, None, 0, st)
            if wg is not None:
                self._wg_pos = (nw_, ng_)
            nleft = cbn[1].cpu().numpy().astype(np.int64)     # one D2H sync, behind the scatter
            ranges = {z["slot"]: (int(starts[z["slot"]]), int(starts[z["slot"]] + nleft[z["slot"]]),
                                  int(ends[z["slot"]])) for z in nodes}
            # child slot ids follow the order of new_nodes built by the caller (left, right per split)
            return new_p2r, new_pn, ranges
        # CPU path
        new_p2r = pos2row.clone()
        new_pn = torch.full_like(pos_node, -1)
        ranges = {}
        bins = self._codes()
        for z in nodes:
            s_ = z["slot"]
            lo, hi = z["start"], z["end"]
            if split_feat[s_] < 0:
                ranges[s_] = (lo, lo, hi)
                continue
            rows = pos2row[lo:hi].long()
            f = int(split_feat[s_])
            b = bins[rows % d.n, f].long()
            if d.is_cat[f]:
                words = torch.from_numpy(cat_left[s_].astype(np.int64))
                left = ((words[b >> 5] >> (b & 31)) & 1) == 1
            else:
                left = b <= int(split_bin[s_])
            lrows, rrows = rows[left], rows[~left]
            new_p2r[lo: lo + lrows.numel()] = lrows.int()
            new_p2r[lo + lrows.numel(): hi] = rrows.int()
            new_pn[lo: lo + lrows.numel()] = child_slots[s_][0]
            new_pn[lo + lrows.numel(): hi] = child_slots[s_][1]
            ranges[s_] = (lo, lo + lrows.numel(), hi)
        return new_p2r, new_pn, ranges

    # ------------------------------------------------------------------------------------
    def apply_tree(self, tree: Tree, data: BinnedData, pred: torch.Tensor, scale: float, set_mode: bool):
        if data.device.type == "cuda":
            from ..ops import _native as nat
            feat, thr, cl, val = tree.device_arrays(data.device)
            ic = torch.from_numpy(data.is_cat.astype(np.uint8)).to(data.device)
            nat.call_hip("shifu_gbdt_apply_tree", data.kbins, data.group_stride, None, feat, thr, cl, val, ic,
                         pred, float(scale), int(set_mode), None, data.n, tree.max_nodes, nat.stream_of(pred))
        else:
            v = torch.from_numpy(tree.predict_bins(data.codes().numpy(), data.is_cat)).float()
            if set_mode:
                pred.copy_(v)
            else:
                pred.add_(scale * v)

    def _residual(self, pred, data: BinnedData, out):
        """out = -dLoss/dpred; returns (sum s*err, sum s) global."""
        loss = LOSS_IDS[self.cfg.loss]
        err = torch.zeros(2, dtype=torch.float64, device=pred.device)
        if pred.device.type == "cuda":
            from ..ops import _native as nat
            nat.call_hip("shifu_gbdt_residual", pred.data_ptr(), data.y.data_ptr(),
                         None if data.sig is None else data.sig.data_ptr(), out.data_ptr(), err.data_ptr(),
                         data.n, loss, nat.stream_of(pred))
        else:
            p, y = pred, data.y
            s = data.sig if data.sig is not None else torch.ones_like(y)
            if loss == 1:
                gr, e = p - y, (p - y) ** 2
            elif loss == 2:
                gr, e = torch.where(y < p, torch.ones_like(p), -torch.ones_like(p)), (y - p).abs()
            elif loss == 3:
                gr = (2 - 4 * y) / torch.exp(4 * y * p - 2 * p)
                e = torch.log1p(1 + torch.exp(2 * p - 4 * p * y))
            else:
                gr, e = 2 * (p - y), (p - y) ** 2
            out.copy_(-gr)
            err[0] = (s.double() * e.double()).sum()
            err[1] = s.double().sum()
        dist.all_reduce_(err)
        e = err.cpu().numpy()                      # one device-to-host copy
        return float(e[0] / max(e[1], 1e-12))

    # ------------------------------------------------------------------------------------
    def train(self, n_trees: int | None = None, callback=None):
        c = self.cfg
        n_trees = c.tree_num if n_trees is None else n_trees
        d = self.data
        # pseudo-residual buffers persist across train() calls (incremental boosting: train(1) per round)
        if getattr(self, "_out", None) is None:
            self._out = torch.zeros(d.n, dtype=torch.float32, device=self.dev)
            self._vout = None if self.valid is None else \
                torch.zeros(self.valid.n, dtype=torch.float32, device=self.valid.device)
        out, vout = self._out, self._vout
        for _ in range(n_trees):
            tid = len(self.trees)
            t_tree = time.perf_counter()
            rows0 = self.hist_rows_total
            self._reseed_rows(tid)
            if c.is_gbt:
                w = self._weights_for_tree()
                if tid == 0:
                    g = d.y
                else:
                    g = out
                scale = 1.0 if tid == 0 else c.learning_rate
                fused = (self.gpu and not (tid > 0 and c.dropout_rate > 0.0)
                         and os.environ.get("SHIFU_GBT_FUSED_PRED", "1") != "0")
                if fused:            # pred += scale * leaf value inside the partition passes
                    if tid == 0:
                        self.pred.zero_()
                    self._fuse = (self.pred, scale)
                    self._leaf_done = False
                try:
                    tree = self.grow_tree(g, w, scale, tid)
                finally:
                    self._fuse = None
                t0 = time.perf_counter()
                with trace_range("gbdt.apply_residual"):
                    keep = None
                    if tid > 0 and c.dropout_rate > 0.0:
                        # DTWorker :634-638: each row skips this tree's update with prob. DropoutRate
                        keep = (torch.rand(d.n, device=self.dev, generator=self.tgen) >= c.dropout_rate).float()
                        before = self.pred.clone()
                    if not fused or not self._leaf_done:      # (max_depth 1: no level pass ran)
                        self.apply_tree(tree, d, self.pred, tree.weight, tid == 0)
                    if keep is not None:
                        self.pred.copy_(before + (self.pred - before) * keep)
                    if self.valid is not None:
                        self.apply_tree(tree, self.valid, self.vpred, tree.weight, tid == 0)
                    self.timings["apply"] += time.perf_counter() - t0
                    terr = self._residual(self.pred, d, out)
                    verr = self._residual(self.vpred, self.valid, vout) if self.valid is not None else float("nan")
            else:
                if not self._pending:
                    # RF: the next trees grow together (their subsample weights drawn in tree order,
                    # so the batch equals growing them one by one)
                    t0 = time.perf_counter()
                    b = self._forest_batch(max(1, c.tree_num - tid))
                    ws = []
                    for k in range(b):          # per-tree streams: the batch == one-by-one growth
                        self._reseed_rows(tid + k)
                        ws.append(self._weights_for_tree())
                    self._pending = self.grow_forest(d.y, ws, 1.0, list(range(tid, tid + b)))
                    self.timings["forest"] = self.timings.get("forest", 0.0) + time.perf_counter() - t0
                tree = self._pending.pop(0)
                self.apply_tree(tree, d, self.pred, 1.0, False)
                if self.valid is not None:
                    self.apply_tree(tree, self.valid, self.vpred, 1.0, False)
                terr, verr = self._rf_errors(tree, tid)
            self.trees.append(tree)
            self.train_errors.append(terr)
            self.valid_errors.append(verr)
            st = self.last_tree_stats if c.is_gbt else None
            self.last_tree_stats = {"tree": tid, "ms": (time.perf_counter() - t_tree) * 1e3,
                                    "hist_rows": self.hist_rows_total - rows0,
                                    "allreduce_ms": self._allreduce_ms(),
                                    "levels": (st or {}).get("levels", [])}
            if callback:
                callback(tid, tree, terr, verr)
        return self.trees

    def _row_error(self, p: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Per-row ``Loss.computeError`` (J/core/dtrain/dt/Loss.java and subclasses)."""
        loss = LOSS_IDS[self.cfg.loss]
        p, y = p.double(), y.double()
        if loss == 2:
            return (y - p).abs()
        if loss == 3:
            return torch.log1p(1 + torch.exp(2 * p - 4 * p * y))
        return (p - y) ** 2

    def _rf_errors(self, tree: Tree, tid: int):
        """RF errors as DTWorker.doCompute accumulates them (J/core/dtrain/dt/DTWorker.java:582-751):
        every tree scores every row with its own leaf ``predict``; an in-bag row adds
        bag-weight * significance * error to the training error, an out-of-bag row (bag weight 0)
        adds significance * error to the validation error, as does every validation-set row.  The
        sums are cumulative over the trees (the reference re-scores all trees each iteration)."""
        d = self.data
        self._reseed_rows(tid)                    # this tree's bag weights (same stream as its growth)
        sub, _ = self._subsample()
        p = torch.empty(d.n, dtype=torch.float32, device=self.dev)
        self.apply_tree(tree, d, p, 1.0, True)
        e = self._row_error(p, d.y)
        sig = d.sig.double() if d.sig is not None else torch.ones(d.n, dtype=torch.float64, device=self.dev)
        acc = torch.zeros(6, dtype=torch.float64, device=self.dev)
        if sub is None:
            acc[0], acc[1] = (sig * e).sum(), sig.sum()
        else:
            sb = sub.double()
            inb = sb > 0
            acc[0], acc[1] = (sb * sig * e)[inb].sum(), (sb * sig)[inb].sum()
            acc[2], acc[3] = (sig * e)[~inb].sum(), sig[~inb].sum()
        if self.valid is not None:
            v = self.valid
            pv = torch.empty(v.n, dtype=torch.float32, device=v.device)
            self.apply_tree(tree, v, pv, 1.0, True)
            sv = v.sig.double() if v.sig is not None else torch.ones(v.n, dtype=torch.float64, device=v.device)
            acc[4], acc[5] = (sv * self._row_error(pv, v.y)).sum().to(self.dev), sv.sum().to(self.dev)
        dist.all_reduce_(acc)
        self._rf_acc = acc if getattr(self, "_rf_acc", None) is None else self._rf_acc + acc
        a = self._rf_acc.cpu().numpy()
        terr = float(a[0] / a[1]) if a[1] > 0 else float("nan")
        verr = float((a[2] + a[4]) / (a[3] + a[5])) if (a[3] + a[5]) > 0 else float("nan")
        self.oob_error = float(a[2] / a[3]) if a[3] > 0 else float("nan")
        return terr, verr

    def _forest_batch(self, remaining: int) -> int:
        """Trees grown per RF batch: ``SHIFU_RF_BATCH`` (default 8), bounded by int32 positions
        and by ~1/3 of free HBM (each tree needs ~40 B per row of position / weight buffers);
        the minimum over ranks so every rank runs the same collectives."""
        n = max(1, self.data.n)
        b = min(int(os.environ.get("SHIFU_RF_BATCH", "8")), remaining, (2 ** 31 - 1) // n)
        if self.gpu:
            from ..utils.device import free_hbm
            free = free_hbm(self.dev)
            b = min(b, int(free // 3 // (40 * n)))
        t = torch.tensor([max(1, b)], dtype=torch.int64, device=self.dev)
        dist.all_reduce_(t, "min")
        return int(t.item())

    # ---- checkpoint / resume (DTMaster.doCheckPoint :637-669 / recoverMasterStatus :1118-1154;
    #      worker-side recoverGBTData :1452-1488 = replay the trees over the resident rows) -----------
    def state_dict(self) -> dict:
        def enc(t):
            return {"max_depth": t.max_depth, "weight": t.weight, "feat": torch.from_numpy(t.feat),
                    "thr": torch.from_numpy(t.thr), "cat_left": torch.from_numpy(t.cat_left.view(np.int32)),
                    "value": torch.from_numpy(t.value), "wgt_cnt": torch.from_numpy(t.wgt_cnt),
                    "class_value": torch.from_numpy(t.class_value), "classification": bool(t.classification),
                    "gain": torch.from_numpy(t.gain), "exists": torch.from_numpy(t.exists),
                    "features_used": list(map(int, t.features_used))}
        trees = [enc(t) for t in self.trees]
        return {"trees": trees, "pending": [enc(t) for t in self._pending], "train_errors": list(self.train_errors), "valid_errors": list(self.valid_errors),
                "rng": self.rng.bit_generator.state}

    def load_state_dict(self, st: dict) -> None:
        def dec(d):
            t = Tree(int(d["max_depth"]), float(d["weight"]))
            t.feat, t.thr = d["feat"].numpy().copy(), d["thr"].numpy().copy()
            t.cat_left = d["cat_left"].numpy().copy().view(np.uint32)
            t.value, t.wgt_cnt = d["value"].numpy().copy(), d["wgt_cnt"].numpy().copy()
            t.gain, t.exists = d["gain"].numpy().copy(), d["exists"].numpy().copy()
            t.features_used = list(d["features_used"])
            if "class_value" in d:
                t.class_value = d["class_value"].numpy().copy()
                t.classification = bool(d["classification"])
            return t
        self.trees = [dec(d) for d in st["trees"]]
        self._pending = [dec(d) for d in st.get("pending", [])]
        self.train_errors, self.valid_errors = list(st["train_errors"]), list(st["valid_errors"])
        self.rng.bit_generator.state = st["rng"]       # row streams: _reseed_rows(tree index)
        self._replay()

    def predict_class(self, data: BinnedData) -> torch.Tensor:
        """Multi-class RF: majority vote of the trees' class values (ties -> lowest class)."""
        C = self.cfg.n_classes
        votes = torch.zeros(data.n, C, dtype=torch.float32, device=data.device)
        cv = torch.empty(data.n, dtype=torch.float32, device=data.device)
        for t in self.trees:
            _apply_classes(self, t, data, cv)
            votes.scatter_add_(1, cv.round().long().clamp(0, C - 1)[:, None], torch.ones_like(cv)[:, None])
        return votes.argmax(1).float()

    def continue_from(self, trees: list) -> None:
        """GBT continuous training (DTMaster.init :1081-1104): start from an existing model's trees
        (first tree weight 1.0, the others their learning rate); predictions and pseudo-residuals
        are replayed over the shard, and the next tree is tree ``len(trees)`` at the current
        learning rate."""
        self.trees = list(trees)
        self._pending = []
        self._replay()

    def _replay(self) -> None:
        # replay predictions and residuals
        self.pred = self.predict(self.data) * (len(self.trees) if not self.cfg.is_gbt and self.trees else 1)
        if self.valid is not None:
            self.vpred = self.predict(self.valid) * (len(self.trees) if not self.cfg.is_gbt and self.trees else 1)
        self._out = torch.zeros(self.data.n, dtype=torch.float32, device=self.dev)
        self._vout = None if self.valid is None else torch.zeros(self.valid.n, dtype=torch.float32,
                                                                   device=self.valid.device)
        if self.cfg.is_gbt and self.trees:
            self._residual(self.pred, self.data, self._out)
        if not self.cfg.is_gbt:          # cumulative in-bag / out-of-bag error sums
            self._rf_acc = None
            for i, t in enumerate(self.trees):
                self._rf_errors(t, i)

    def predict(self, data: BinnedData) -> torch.Tensor:
        if self.cfg.is_multiclass:
            return self.predict_class(data)
        p = torch.zeros(data.n, dtype=torch.float32, device=data.device)
        for i, t in enumerate(self.trees):
            if self.cfg.is_gbt:
                self.apply_tree(t, data, p, t.weight, i == 0)
            else:
                self.apply_tree(t, data, p, 1.0, False)
        if not self.cfg.is_gbt and self.trees:
            p /= len(self.trees)
        return p


def _apply_classes(tr: "TreeTrainer", t: Tree, data: BinnedData, out: torch.Tensor) -> None:
    """out = the tree's class value per row (classification leaves)."""
    if data.device.type == "cuda":
        from ..ops import _native as nat
        feat, thr, cl, val = t.device_arrays(data.device, classes=True)
        ic = torch.from_numpy(data.is_cat.astype(np.uint8)).to(data.device)
        nat.call_hip("shifu_gbdt_apply_tree", data.kbins, data.group_stride, None, feat, thr, cl, val, ic,
                     out, 1.0, 1, None, data.n, t.max_nodes, nat.stream_of(out))
    else:
        out.copy_(torch.from_numpy(t.predict_bins(data.codes().numpy(), data.is_cat, classes=True)).float())


def _group_pairs(items: np.ndarray) -> np.ndarray:
    """[n_pairs][2] item ids of groups (2j, 2j + 1) with the same node and row range (-1 where a
    group has no partner), in item order.  _make_items emits the groups of one (node, chunk) in
    ascending order and consecutively, so a partner is always the next item: O(n), no sort (a
    row-wise np.unique took milliseconds per level on the host, between two GPU launches)."""
    n = len(items)
    if n == 0:
        return np.zeros((0, 2), np.int32)
    slot, lo, hi, grp = items[:, 0], items[:, 1], items[:, 2], items[:, 3]
    nxt = np.zeros(n, dtype=bool)                 # item i is paired with item i + 1
    nxt[:-1] = (((grp[:-1] & 1) == 0) & (grp[1:] == grp[:-1] + 1) & (slot[1:] == slot[:-1])
                & (lo[1:] == lo[:-1]) & (hi[1:] == hi[:-1]))
    taken = np.zeros(n, dtype=bool)
    taken[1:] = nxt[:-1]                          # the partner (second) of a pair
    first = np.flatnonzero(~taken)                # every pair starts at an item not taken
    pairs = np.full((len(first), 2), -1, np.int32)
    even = (grp[first] & 1) == 0
    pairs[even, 0] = first[even]
    pairs[~even, 1] = first[~even]
    pairs[nxt[first], 1] = first[nxt[first]] + 1
    return pairs


def _zm(z) -> int:
    """Rows of a node: exact (end - start) or the estimate "m" of a node whose range is still on
    the device."""
    return max(0, int(z["m"])) if "m" in z else max(0, z["end"] - z["start"])


def _slot_key(z):
    """Slot order of a level's nodes: built first (one contiguous all-reduce), then by tree, id."""
    return (not z["built"], z["tree"], z["id"])


def _host_device_pointer(t: torch.Tensor) -> int:
    """Device address of a pinned host tensor (hipHostGetDevicePointer on the HIP runtime torch
    already loaded)."""
    import ctypes
    if not t.is_pinned():
        raise RuntimeError("host-resident bins must be pinned")
    lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    out = ctypes.c_void_p()
    rc = lib.hipHostGetDevicePointer(ctypes.byref(out), ctypes.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not out.value:
        raise RuntimeError(f"hipHostGetDevicePointer failed ({rc}): cannot map host-resident bins")
    return int(out.value)


W_BITS, G_BITS = 16, 23     # per-row fixed-point magnitude bounds (packed histogram fields)
# root level of a single-tree (non-forest) build: u32 histogram modes, w*g on a grid 2^3 coarser
# (gbdt_kernels.hip GSH32); SHIFU_GBDT_ROOT_U32=0 keeps the packed u64 kernel everywhere
ROOT_U32 = os.environ.get("SHIFU_GBDT_ROOT_U32", "1") != "0"
ROOT_GSH32 = 3               # = gbdt_kernels.hip GSH32
# root sum w*g over whole quad records when there is no [G][N][32] copy (SHIFU_GBDT_ROOT_QUAD=0:
# the per-group items); SHIFU_GBDT_ROOT_G32=0 never makes the copy
ROOT_QUAD = os.environ.get("SHIFU_GBDT_ROOT_QUAD", "1") != "0"
ROOT_G32 = os.environ.get("SHIFU_GBDT_ROOT_G32", "1") != "0"
# final-level prediction update in row windows of LEAF_W rows, LEAF_Y blocks per window
LEAF_WINDOW = os.environ.get("SHIFU_GBDT_LEAF_WINDOW", "1") != "0"
# below-root histograms over 64-feature half records (gbdt_hist64_kernel); 0 = 32-feature items
HIST64 = os.environ.get("SHIFU_GBDT_HIST64", "1") != "0"
# ... on levels whose built nodes average at least this many rows.  With 2048 items per level the
# 1024-thread blocks (one per CU) lost on short row ranges (2M rows: 1.9 vs 1.0 ms); with 4096
# items they win or tie down to 2.8M rows per node (balanced levels 5 / 6: 13.2 / 14.0 vs 14.5 /
# 14.8 ms) and tie on the favourable labels' small levels (profiles/r5/gbdt/hist64_threshold_r5.txt)
# (r6, with the static-slot prefetch and v_perm addressing: 500K rows per built node -- favourable
# levels 3 / 5 / 6 at 2.26 / 3.33 / 4.07 vs 2.36 / 3.51 / 4.22 ms, balanced unchanged;
# profiles/r6/gbdt/hist64_threshold_r6.txt)
HIST64_MIN_NODE_ROWS = int(os.environ.get("SHIFU_GBDT_HIST64_MIN_NODE_ROWS", "500000"))
# split decisions on the device, queued ahead of the partition (one host sync per level, which
# the partition hides); SHIFU_GBDT_DEV_DECIDE=0: host decisions between the split scan and the
# partition (two syncs per level).  Trees with MaxLeaves, native multi-class trees and levels of
# more than 512 nodes always take the host path.
DEV_DECIDE = os.environ.get("SHIFU_GBDT_DEV_DECIDE", "1") != "0"
DECIDE_CHECK = os.environ.get("SHIFU_GBDT_DECIDE_CHECK", "0") == "1"
# single-tree builds move (w, g) with the rows in the partition scatter so the histograms read
# them in position order; SHIFU_GBDT_WG_POS=0: the histograms gather w[row], g[row] instead
WG_POS = os.environ.get("SHIFU_GBDT_WG_POS", "1") != "0"
# device-decision levels: the partition finds a position's node by searching the level's node
# ranges (sorted by start) instead of reading / writing a per-position node array (8-12 B per
# position per level less); SHIFU_GBDT_RANGE_NODES=0 keeps the array
RANGE_NODES = os.environ.get("SHIFU_GBDT_RANGE_NODES", "1") != "0"
LEAF_W = int(os.environ.get("SHIFU_GBDT_LEAF_W", str(1 << 16)))
LEAF_Y = int(os.environ.get("SHIFU_GBDT_LEAF_Y", "128"))   # 0.96 vs 2.13 ms with 16 (tools/leafwin_sweep.sh)
# what the histograms really hold (bench label): per-row w and w*g quantised to fixed point on
# power-of-two grids (|w*g| < 2^23 of the grid, the root's u32 w*g mode 2^3 coarser), summed
# exactly in int64 (so every rank and every run finds the same splits)
HIST_DTYPE_LABEL = "int64 fixed-point hist (w 16-bit, w*g 23-bit grid; root w*g 20-bit)/uint8-bins"
ROOT_G_DIV = 1 << ROOT_GSH32


def _pack_scale(max_abs: float, bits: int, margin: float = 1.0) -> float:
    """Largest 2^S with max_abs * 2^S <= 2^bits - margin (so the rounded value stays < 2^bits)."""
    if not max_abs > 0 or not math.isfinite(max_abs):
        return 1.0
    return float(2.0 ** min(60, math.floor(math.log2((2.0 ** bits - margin) / max_abs))))


def _gain_py(imp, lw, ls, rw, rs):
    c, s = lw + rw, ls + rs
    if imp == 1:
        dd = rw * ls - lw * rs
        return dd * dd / (lw * rw * c)
    if imp in (2, 3):
        def ent(nn, p1):
            if nn <= 0:
                return 0.0
            r1 = p1 / nn
            r0 = 1 - r1
            if imp == 3:
                return -(r1 * r1 + r0 * r0)
            e = 0.0
            if r1 > 0:
                e -= r1 * math.log2(r1)
            if r0 > 0:
                e -= r0 * math.log2(r0)
            return e
        return ent(c, s) - (lw / c) * ent(lw, ls) - (rw / c) * ent(rw, rs)
    return (ls * ls / lw + rs * rs / rw - s * s / c) / c


# ------------------------------------------------------------------------------------------
# smoke + bench hooks
# ------------------------------------------------------------------------------------------
def synthetic_binned(n, f, device, seed=0, n_bins=256, labels="favourable"):
    """uint8 codes (quad-blocked [Q, n, 128]) generated chunk-wise on the device (no int32 staging of the whole
    matrix) + labels.  ``favourable``: a hidden rule on the first two features (later splits peel off
    small minorities: few rows histogrammed below the root).  ``balanced``: a dense random linear
    rule over ALL codes thresholded at its median (the codes are iid uniform, so the median of the
    symmetric score is its mean): every split lands near a feature's median bin and the smaller
    child of each node holds about half its rows -- the worst case for the histogram work."""
    g = torch.Generator(device=device).manual_seed(seed)
    wv = None
    if labels == "balanced":
        wv = torch.randn(f, generator=g, device=device, dtype=torch.float32)
        thr = float(wv.sum()) * (n_bins - 1) / 2.0
    ng = (f + FG - 1) // FG
    codes = torch.zeros((f + QF - 1) // QF, n, QF, dtype=torch.uint8, device=device)
    y = torch.empty(n, dtype=torch.float32, device=device)
    step = 1 << 21
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        blk = torch.randint(0, n_bins, (r1 - r0, f), generator=g, device=device, dtype=torch.int32)
        for gi in range(ng):
            c0, c1 = gi * FG, min(f, (gi + 1) * FG)
            o = (gi % (QF // FG)) * FG
            codes[gi // (QF // FG), r0:r1, o: o + c1 - c0] = blk[:, c0:c1].to(torch.uint8)
        if wv is not None:
            sc = blk.float() @ wv
            y[r0:r1] = (sc + 0.05 * sc.abs().mean() * torch.randn(r1 - r0, generator=g, device=device) > thr).float()
        else:
            x0 = blk[:, 0].float() / n_bins
            x1 = blk[:, 1].float() / n_bins
            y[r0:r1] = ((x0 + 0.5 * x1 + 0.1 * torch.rand(r1 - r0, generator=g, device=device)) > 0.8).float()
    nb = np.full(f, n_bins, np.int32)
    return BinnedData(codes, y, None, nb, np.zeros(f, np.uint8), f)


def smoke_gbdt(dev):
    data = synthetic_binned(5000, 40, dev, seed=3, n_bins=64)
    tr = TreeTrainer(TreeConfig("GBT", tree_num=3, max_depth=4, learning_rate=0.1,
                                feature_subset_strategy="ALL"), data)
    tr.train()
    assert tr.train_errors[-1] <= tr.train_errors[0] + 1e-6, tr.train_errors
    return tr.train_errors


def bench_rounds(a, dev, info):
    """GBDT config: 500 trees depth 7, 256-bin histograms, 100M rows x 1000 cols per GPU.
    One step = one boosting round (one tree)."""
    rows = a.rows
    labels = getattr(a, "labels", "favourable")
    data = synthetic_binned(rows, a.cols, dev, seed=11 + info.rank, labels=labels)
    cfg = TreeConfig("GBT", tree_num=500, max_depth=7, learning_rate=0.05,
                     feature_subset_strategy="ALL", min_instances_per_node=5)
    tr = TreeTrainer(cfg, data)
    late = int(getattr(a, "late", 0) or 0)
    for _ in range(a.warmup + late):    # --gbdt-late: time a later window (rounds late+w .. late+w+k)
        tr.train(1)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    if dev.type == "cuda" and getattr(a, "levels", False):
        tr.level_stats = []
    rows0 = tr.hist_rows_total
    t0 = time.perf_counter()
    tr.train(a.steps)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    hist_rows = (tr.hist_rows_total - rows0) / max(1, a.steps)
    levels = None
    if tr.level_stats:               # per level: rows histogrammed, bytes of codes read, ms, TB/s
        agg = {}
        for e in tr.level_stats:
            r = agg.setdefault(e["level"], {"level": e["level"], "rows": 0, "nodes_built": 0, "ms": 0.0})
            r["rows"] += e["rows"]
            r["nodes_built"] += e["nodes_built"]
            r["ms"] += e["ev"][0].elapsed_time(e["ev"][1])
        levels = []
        for lv in sorted(agg):
            r = agg[lv]
            k = a.steps
            gb = r["rows"] * (a.cols + 8) / k / 1e9         # codes + (w, g) per row touched
            levels.append({"level": lv, "rows_per_round": r["rows"] // k, "nodes_built": r["nodes_built"] // k,
                           "ms_per_round": round(r["ms"] / k, 3), "gb_per_round": round(gb, 2),
                           "tb_per_s": round(gb / (r["ms"] / k), 2) if r["ms"] > 0 else None})
        tr.level_stats = None
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")
    dt = float(t.item())
    return {
        "metric": "GBDT rounds/sec (boosting rounds, depth 7, 256 bins)",
        "value": a.steps / dt, "unit": "rounds/s", "n_gpus": info.world_size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": HIST_DTYPE_LABEL,
        "data": f"synthetic uint8 bin codes, {labels} labels "
                + ("(dense linear rule over all codes at its median)" if labels == "balanced"
                   else "(hidden rule on two features)"),
        "labels": labels, "hist_rows_per_round": hist_rows, "late_rounds": late,
        "config": {"model": "GBT 500 trees depth=7 256 bins", "global_batch": rows * info.world_size,
                   "seq_len": None, "n_cols": a.cols, "parallelism": f"dp{info.world_size}"},
        "timings_s": tr.timings, "train_error": tr.train_errors[-1], "levels": levels,
    }
