"""Snapshot graph: the DGL-free replacement of the object built by rgcn/utils.py:100-134.

`build_sub_graph(num_nodes, num_rels, triples, use_cuda, gpu)` keeps the reference
signature and edge semantics bit-exactly:
  * edges in the reference order: src = cat(s, o), dst = cat(o, s), type = cat(r, r + R)
    (rgcn/utils.py:116-118, :125);
  * in-degree over the doubled graph, norm = 1/in_deg with 0 -> 1, fp32 (:110-114);
  * edge norm = norm[dst] * norm[src] (:124); node id = arange(V) (:122);
  * uniq_r / r_len / r_to_e as in r2e (:78-97); each r_to_e span holds the same entity
    SET as the reference (its order there is Python set-iteration order).

On top of the DGL-visible surface (ndata/edata/in_degrees/number_of_nodes/to) the
object carries the device-side work lists the HIP kernels consume:
  * a destination-sorted CSR (stable, so equal destinations keep edge-id order):
    col_src / col_type int32;
  * `chunks` int32[n][4] = {row, edge_begin, edge_end, slot} with at most
    `chunk_edges` edges per chunk, and `fixups` int32[m][4] = {row, slot_begin,
    slot_end, 0} for rows split over several chunks (see csrc/aggregate.hip);
  * `rows` int32[V]: rows with in-degree > 0 first, then the rest (`n_pos` of the
    former), so every 64-row tile of the layer GEMM uses one self-loop weight;
  * the same chunking over the forward relations' r_to_e spans for the relation-context
    mean (an inverse relation's span repeats its forward relation's entities).
Built once per snapshot and cached across epochs: on the device by
csrc/graphbuild.hip when use_cuda (build_sub_graph_device), else with numpy here; both
builds produce the same lists bit for bit (tests/test_gpu_graph.py).
"""
import os

import numpy as np
import torch

DEFAULT_CHUNK_EDGES = None  # adaptive, see chunk_size_for()


def chunk_size_for(num_edges):
    """Edges per work chunk: small snapshots (ICEWS/GDELT: 0.5-3k edges, Zipf in-degrees
    with hubs of hundreds of edges) are latency-bound, so chunks are cut short (16) to
    spread a hub over many waves; large snapshots get up to 1024 edges per wave."""
    return int(min(1024, max(16, num_edges // 4096)))


def r2e(triplets, num_rels):
    """rgcn/utils.py:78-97.  Returns (uniq_r, r_len list of (start, end), r_to_e list)."""
    triplets = np.asarray(triplets, dtype=np.int64).reshape(-1, 3)
    src, rel, dst = triplets[:, 0], triplets[:, 1], triplets[:, 2]
    uniq = np.unique(rel)
    uniq_r = np.concatenate((uniq, uniq + num_rels))
    if len(triplets) == 0:
        return uniq_r, [], []
    order = np.argsort(rel, kind="stable")
    rel_sorted = rel[order]
    starts = np.searchsorted(rel_sorted, uniq, side="left")
    ends = np.searchsorted(rel_sorted, uniq, side="right")
    per_rel = []
    for a, b in zip(starts, ends):
        idx = order[a:b]
        per_rel.append(np.unique(np.concatenate((src[idx], dst[idx]))))
    r_len, e_idx, pos = [], [], 0
    for ents in per_rel + per_rel:  # inverse ids share the forward set (:88-89)
        r_len.append((pos, pos + len(ents)))
        e_idx.append(ents)
        pos += len(ents)
    return uniq_r, r_len, np.concatenate(e_idx).tolist()


FIX_GROUP = 64  # partial slots one fix-up wave sums; longer rows get a first-level group pass


def group_fixups(fixups, nslot, group=FIX_GROUP):
    """Cut fix-ups over more than `group` slots into first-level groups (csrc/aggregate.hip
    k_fixup_groups): {0, b, e, k + 1} sums slots [b, e) into new slot k, and the row's own
    fix-up then sums its groups' slots.  A hub's thousands of chunk partials are thus summed
    by many waves instead of one wave walking them all.  Returns (fixups, nslot)."""
    fixups = np.asarray(fixups, dtype=np.int32).reshape(-1, 4)
    if len(fixups) == 0:
        return fixups, nslot
    k = fixups[:, 2].astype(np.int64) - fixups[:, 1]
    big = k > group
    if not big.any():
        return fixups, nslot
    groups, finals = [], []
    for row, sb, se, _ in fixups[big].tolist():
        ng = (se - sb + group - 1) // group
        for g in range(ng):
            groups.append((0, sb + g * group, min(sb + (g + 1) * group, se), nslot + g + 1))
        finals.append((row, nslot, nslot + ng, 0))
        nslot += ng
    out = np.concatenate([np.asarray(groups, dtype=np.int32).reshape(-1, 4), fixups[~big],
                          np.asarray(finals, dtype=np.int32).reshape(-1, 4)])
    return out, int(nslot)


def _chunk_rows(seg_ptr, seg_rows, chunk_edges):
    """Cut segments [seg_ptr[i], seg_ptr[i+1]) of row seg_rows[i] into chunks."""
    lens = np.diff(seg_ptr)
    nz = lens > 0
    rows, beg, lens = seg_rows[nz], seg_ptr[:-1][nz], lens[nz]
    nchunk = (lens + chunk_edges - 1) // chunk_edges
    total = int(nchunk.sum())
    rep_rows = np.repeat(rows, nchunk)
    rep_beg = np.repeat(beg, nchunk)
    first = np.repeat(np.cumsum(nchunk) - nchunk, nchunk)
    k = np.arange(total) - first
    c_beg = rep_beg + k * chunk_edges
    c_end = np.minimum(c_beg + chunk_edges, np.repeat(beg + lens, nchunk))
    multi = np.repeat(nchunk > 1, nchunk)
    slot = np.full(total, -1, dtype=np.int64)
    slot[multi] = np.arange(int(multi.sum()))
    chunks = np.stack([rep_rows, c_beg, c_end, slot], 1).astype(np.int32)
    long_rows = rows[nchunk > 1]
    ncl = nchunk[nchunk > 1]
    sb = np.cumsum(ncl) - ncl
    fixups = np.stack([long_rows, sb, sb + ncl, np.zeros_like(ncl)], 1).astype(np.int32)
    fixups, nslot = group_fixups(fixups, int(multi.sum()))
    return chunks.reshape(-1, 4), fixups, nslot


class _Frame(dict):
    """dict with DGL's `ndata`/`edata` feel (get/pop/update/[])."""


class SnapshotGraph:
    """One temporal snapshot (see module docstring)."""

    def __init__(self, num_nodes, num_rels, src, dst, etype, uniq_r, r_len, r_to_e,
                 chunk_edges=DEFAULT_CHUNK_EDGES, tile_budget=None):
        V = int(num_nodes)
        self.num_nodes_, self.num_rels = V, int(num_rels)
        self.device = torch.device("cpu")
        E = len(src)
        if V >= 2 ** 31 - 1 or E >= 2 ** 31 - 1:
            raise ValueError("snapshot too large for int32 indices")
        in_deg = np.bincount(dst, minlength=V).astype(np.int64)
        deg_f = in_deg.astype(np.float32)
        deg_f[deg_f == 0] = 1.0
        norm = (np.float32(1.0) / deg_f).astype(np.float32)
        self.src_np, self.dst_np, self.type_np = src, dst, etype
        self.in_deg_np = in_deg
        self.uniq_r = uniq_r
        self.r_len = r_len
        self.r_to_e = r_to_e
        self.ndata = _Frame(id=torch.arange(V, dtype=torch.long).view(-1, 1),
                            norm=torch.from_numpy(norm).view(-1, 1))
        self.edata = _Frame(type=torch.from_numpy(etype.astype(np.int64)),
                            norm=torch.from_numpy((norm[dst] * norm[src]).astype(np.float32)).view(-1, 1))
        # ---- kernel work lists (int32, host) ----
        order = np.argsort(dst, kind="stable")
        rowptr = np.zeros(V + 1, dtype=np.int64)
        np.cumsum(in_deg, out=rowptr[1:])
        self.chunk_edges = int(chunk_edges) if chunk_edges else chunk_size_for(E)
        chunks, fixups, nslot = _chunk_rows(rowptr, np.arange(V), self.chunk_edges)
        col_src_s, col_type_s = src[order], etype[order]
        if len(etype) and int(etype.max()) >= 2 ** 27:
            raise ValueError("relation ids must be < 2^27")
        # fused-layer work (csrc/layer.hip) over all nodes
        self.budget = int(tile_budget) if tile_budget else tile_budget_for(
            E, self.chunk_edges, int(in_deg.max()) if V else 0)
        # small snapshots pack ~32 inline edges per tile (8 per wave = one batch in flight);
        # a row up to the budget still sits alone in its own tile
        self.pack_items = min(32, self.budget) if E <= 65536 else self.budget
        fw = fused_work(np.arange(V), in_deg, rowptr, col_src_s, col_type_s, self.budget, self.pack_items,
                        self.chunk_edges)
        R2 = 2 * self.num_rels
        rel_count = np.zeros(R2, dtype=np.float32)
        rel_start = np.zeros(R2, dtype=np.int64)
        if len(r_len):
            lens = np.array([b - a for a, b in r_len], dtype=np.int64)
            ur = np.asarray(uniq_r, dtype=np.int64)
            rel_count[ur] = lens
            # spans are laid out in uniq_r order; re-express them per relation id
            starts = np.array([a for a, _ in r_len], dtype=np.int64)
            rel_start[ur] = starts
            rel_len = np.zeros(R2, dtype=np.int64)
            rel_len[ur] = lens
            # forward relations only: the inverse id r + R has the same span contents (r2e), so
            # its mean is a copy of r's (hyperbolic_model.relation_context)
            rchunks, rfix, rslot = _chunk_rows_spans(rel_start[:self.num_rels], rel_len[:self.num_rels],
                                                     self.chunk_edges)
        else:
            rchunks, rfix, rslot = np.zeros((0, 4), np.int32), np.zeros((0, 4), np.int32), 0
        self._host_lists = {
            "col_src": col_src_s.astype(np.int32), "col_type": col_type_s.astype(np.int32),
            "chunks": chunks, "fixups": fixups, "norm": norm,
            "rel_idx": np.asarray(r_to_e, dtype=np.int32).reshape(-1),
            "rel_count": rel_count, "rel_chunks": rchunks, "rel_fixups": rfix,
            "rel_start": rel_start.astype(np.int32),
            "rowptr": rowptr.astype(np.int32),
        }
        self._host_lists.update(fw.host)
        self.n_pos, self.n_pos_tiles = fw.n_pos, fw.n_pos_tiles
        self.n_heavy, self.heavy_slots = fw.n_heavy, fw.heavy_slots
        self.n_slots = nslot
        self.rel_slots = rslot
        # relation spans short enough for the GRU kernel's in-kernel mean (csrc/relgru.hip)
        self.rel_max_span = int(rel_count.max()) if R2 else 0
        self.dev = None

    # ---------------------------------------------------------------- DGL-visible surface
    def number_of_nodes(self):
        return self.num_nodes_

    def number_of_edges(self):
        return int(len(self.src_np))

    def in_degrees(self, v=None):
        deg = torch.from_numpy(self.in_deg_np).to(self.device)
        if v is None:
            return deg
        idx = torch.as_tensor(list(v) if isinstance(v, range) else v, dtype=torch.long, device=self.device)
        return deg[idx]

    def edges(self):
        return torch.from_numpy(self.src_np), torch.from_numpy(self.dst_np)

    def to(self, device):
        """Move the graph (node/edge data and kernel work lists) to `device`.
        Accepts the reference's gpu ids (int), strings or torch.device."""
        if isinstance(device, int):
            device = torch.device("cuda", device) if device >= 0 else torch.device("cpu")
        device = torch.device(device)
        if device == self.device:
            return self
        g = object.__new__(type(self))
        g.__dict__.update(self.__dict__)
        g.device = device
        g.ndata = _Frame({k: v.to(device) for k, v in self.ndata.items()})
        g.edata = _Frame({k: v.to(device) for k, v in self.edata.items()})
        g.dev = {k: torch.from_numpy(v).to(device) for k, v in self._host.items()} if device.type == "cuda" else None
        return g

    @property
    def _host(self):
        """Host copies of the kernel work lists (int32 / fp32 numpy)."""
        return self._host_lists

    def transposed(self):
        """Edge lists of the backward passes (regcn_snapshot_transpose_i32), built on first use
        and cached: csr_dst (destination of each CSR position), CSR positions sorted by
        source (sptr, sp) and by relation type (tptr, tp)."""
        t = self.__dict__.get("_transposed")
        if t is not None:
            return t
        import ctypes
        from . import _lib
        wk = self.work()
        dev = wk["rowptr"].device
        V, E, R2 = self.num_nodes_, int(wk["col_src"].shape[0]), 2 * self.num_rels
        ws = torch.empty(int(_lib.lib().regcn_transpose_workspace_bytes(E, V, R2)), dtype=torch.uint8, device=dev)
        t = {"csr_dst": torch.empty(max(E, 1), dtype=torch.int32, device=dev),
             "sptr": torch.empty(V + 1, dtype=torch.int32, device=dev),
             "sp": torch.empty(max(E, 1), dtype=torch.int32, device=dev),
             "tptr": torch.empty(R2 + 1, dtype=torch.int32, device=dev),
             "tp": torch.empty(max(E, 1), dtype=torch.int32, device=dev)}
        a = _lib.TransposeDesc()
        a.V, a.E, a.R2 = V, E, R2
        a.rowptr = ctypes.c_void_p(wk["rowptr"].data_ptr())
        a.col_src = ctypes.c_void_p(wk["col_src"].data_ptr()) if E else None
        a.col_type = ctypes.c_void_p(wk["col_type"].data_ptr()) if E else None
        a.workspace, a.ws_bytes = ctypes.c_void_p(ws.data_ptr()), ws.numel()
        for k, v in t.items():
            setattr(a, k, ctypes.c_void_p(v.data_ptr()))
        _lib.call_desc("regcn_snapshot_transpose_i32", a)
        _lib.publish()  # cached: read next by whichever stream asks
        self.__dict__["_transposed"] = t
        return t

    def row_type_cols(self):
        """(col_src, col_type) with each destination row's edges in relation-type order
        (regcn_snapshot_row_type_order_i32), built on first use and cached: the edge lists
        the chunked Lorentz aggregation reads (a row's same-type run reuses the type's
        relation row and W blocks from L1)."""
        t = self.__dict__.get("_row_type")
        if t is not None:
            return t
        from . import _lib
        wk = self.work()
        dev = wk["rowptr"].device
        V, E, R2 = self.num_nodes_, int(wk["col_src"].shape[0]), 2 * self.num_rels
        if E == 0:
            t = (wk["col_src"], wk["col_type"])
        else:
            ws = torch.empty(int(_lib.lib().regcn_row_type_order_workspace_bytes(E, V, R2)), dtype=torch.uint8,
                             device=dev)
            t = (torch.empty(E, dtype=torch.int32, device=dev), torch.empty(E, dtype=torch.int32, device=dev))
            _lib.call("regcn_snapshot_row_type_order_i32", V, E, R2, _lib.iptr(wk["rowptr"]), _lib.iptr(wk["col_src"]),
                      _lib.iptr(wk["col_type"]), _lib.iptr(t[0]), _lib.iptr(t[1]), ws.data_ptr(), ws.numel(),
                      _lib.stream())
            _lib.publish()  # cached: read next by whichever stream asks
        self.__dict__["_row_type"] = t
        return t

    def row_src_cols(self):
        """col_src with each destination row's edges in ascending source order
        (regcn_snapshot_row_src_order_i32), built on first use and cached: the source half of
        the union hub-row aggregation gathers a row's duplicate sources once."""
        t = self.__dict__.get("_row_src")
        if t is not None:
            return t
        from . import _lib
        wk = self.work()
        dev = wk["rowptr"].device
        V, E = self.num_nodes_, int(wk["col_src"].shape[0])
        if E == 0:
            t = wk["col_src"]
        else:
            ws = torch.empty(int(_lib.lib().regcn_row_src_order_workspace_bytes(E, V)), dtype=torch.uint8, device=dev)
            t = torch.empty(E, dtype=torch.int32, device=dev)
            _lib.call("regcn_snapshot_row_src_order_i32", V, E, _lib.iptr(wk["rowptr"]), _lib.iptr(wk["col_src"]),
                      _lib.iptr(t), ws.data_ptr(), ws.numel(), _lib.stream())
            _lib.publish()  # cached: read next by whichever stream asks
        self.__dict__["_row_src"] = t
        return t

    # fused-layer items in (row, source) order: on for snapshots with at least this many
    # inline items (config 5), where a row's duplicate sources are common; the dataset-sized
    # snapshots keep CSR item order (the phase launches read the same lists).  A graph's
    # `item_src_runs` attribute (True / False) overrides the size rule.
    ITEM_SRC_RUNS_MIN_ITEMS = 1 << 20
    item_src_runs = None

    def use_item_src_runs(self):
        if self.item_src_runs is not None:
            return bool(self.item_src_runs)
        return int(self.work()["item_src"].numel()) >= self.ITEM_SRC_RUNS_MIN_ITEMS

    def item_src_cols(self):
        """(item_src, item_tl) with each row's inline items in ascending source order
        (regcn_snapshot_item_src_order_i32), built on first use and cached: with
        regcn_layer_desc.item_src_runs the fused gather loads a row's duplicate sources once."""
        t = self.__dict__.get("_item_src")
        if t is not None:
            return t
        from . import _lib
        wk = self.work()
        dev = wk["rowptr"].device
        n_items, n_tiles = int(wk["item_src"].numel()), int(self.n_pos_tiles)
        if n_items == 0:
            t = (wk["item_src"], wk["item_tl"])
        else:
            ws = torch.empty(int(_lib.lib().regcn_item_src_order_workspace_bytes(n_items, self.num_nodes_)),
                             dtype=torch.uint8, device=dev)
            t = (torch.empty(n_items, dtype=torch.int32, device=dev), torch.empty(n_items, dtype=torch.int32, device=dev))
            _lib.call("regcn_snapshot_item_src_order_i32", self.num_nodes_, n_tiles, n_items, _lib.iptr(wk["tiles"]),
                      _lib.iptr(wk["item_ptr"]), _lib.iptr(wk["item_src"]), _lib.iptr(wk["item_tl"]), _lib.iptr(t[0]),
                      _lib.iptr(t[1]), ws.data_ptr(), ws.numel(), _lib.stream())
            _lib.publish()  # cached: read next by whichever stream asks
        self.__dict__["_item_src"] = t
        return t

    def item_type_cols(self):
        """(item_src, item_tl) with each row's inline items in ascending relation-type order
        (regcn_snapshot_item_type_order_i32), built on first use and cached: with
        regcn_layer_desc.item_crel the gather sums a row's same-type item weights and applies the
        relation rows as one MFMA product per tile."""
        t = self.__dict__.get("_item_type")
        if t is not None:
            return t
        from . import _lib
        wk = self.work()
        dev = wk["rowptr"].device
        n_items, n_tiles = int(wk["item_src"].numel()), int(self.n_pos_tiles)
        if n_items == 0:
            t = (wk["item_src"], wk["item_tl"])
        else:
            ws = torch.empty(int(_lib.lib().regcn_item_src_order_workspace_bytes(n_items, self.num_nodes_)),
                             dtype=torch.uint8, device=dev)
            t = (torch.empty(n_items, dtype=torch.int32, device=dev), torch.empty(n_items, dtype=torch.int32, device=dev))
            _lib.call("regcn_snapshot_item_type_order_i32", self.num_nodes_, 2 * self.num_rels, n_tiles, n_items,
                      _lib.iptr(wk["tiles"]), _lib.iptr(wk["item_ptr"]), _lib.iptr(wk["item_src"]),
                      _lib.iptr(wk["item_tl"]), _lib.iptr(t[0]), _lib.iptr(t[1]), ws.data_ptr(), ws.numel(),
                      _lib.stream())
            _lib.publish()
        self.__dict__["_item_type"] = t
        return t

    def work(self):
        """Device work lists (raises on a CPU graph: the HIP path has no CPU fallback)."""
        if self.dev is None:
            raise ValueError("SnapshotGraph must be moved to a HIP device (g.to('cuda')) before message passing")
        return self.dev


class FusedWork:
    """Work lists of the fused layer kernel over a set of destination rows (all nodes of
    a snapshot, or one rank's rows under the owner partition, parallel.py)."""

    def __init__(self, host, n_pos, n_pos_tiles, n_heavy, heavy_slots):
        self.host, self.n_pos, self.n_pos_tiles = host, n_pos, n_pos_tiles
        self.n_heavy, self.heavy_slots = n_heavy, heavy_slots


def fused_work(nodes, in_deg, rowptr, col_src_s, col_type_s, budget, pack_items, chunk_edges):
    """rows: the nodes with in-degree > 0 sorted by in-degree (descending, stable), then the
    rest; tiles packed under `pack_items` inline edges; rows over `budget` pre-aggregated
    (heavy chunks); per-tile flattened in-edge items (item_src, item_tl = type << 4 |
    tile-local row, item_ptr)."""
    nodes = np.asarray(nodes, dtype=np.int64)
    deg = in_deg[nodes]
    pos = nodes[deg > 0]
    pos = pos[np.argsort(-in_deg[pos], kind="stable")]
    zero = nodes[deg == 0]
    heavy = pos[in_deg[pos] > budget]
    inl = np.where(in_deg[pos] > budget, 0, in_deg[pos])
    tiles = _pack_tiles(inl, pack_items)
    hchunks, hfixups, hslot = _chunk_spans(rowptr[heavy], in_deg[heavy], heavy, chunk_edges)
    n_items = int(inl.sum())
    first = np.cumsum(inl) - inl
    perm = np.arange(n_items, dtype=np.int64) + np.repeat(rowptr[pos] - first, inl)
    if len(tiles):
        local = np.arange(len(pos)) - np.repeat(tiles[:, 0].astype(np.int64), tiles[:, 1].astype(np.int64))
    else:
        local = np.zeros(0, np.int64)
    item_src = col_src_s[perm].astype(np.int32)
    item_tl = ((col_type_s[perm].astype(np.int64) << 4) | np.repeat(local, inl)).astype(np.int32)
    item_ptr = np.zeros(len(tiles) + 1, dtype=np.int64)
    if len(tiles):
        item_ptr[1:] = np.cumsum(np.add.reduceat(inl, tiles[:, 0]))
    host = {"rows": np.concatenate([pos, zero]).astype(np.int32), "tiles": tiles, "heavy_chunks": hchunks,
            "heavy_fixups": hfixups, "item_src": item_src, "item_tl": item_tl,
            "item_ptr": item_ptr.astype(np.int32)}
    return FusedWork(host, int(len(pos)), int(len(tiles)), int(len(heavy)), hslot)


def tile_budget_for(num_edges, chunk_edges, max_deg=0):
    """In-edges one fused-layer tile gathers inline (4 waves share them, 8 in flight per
    wave).  Small snapshots take every row up to 256 in-edges inline: a hub tile then runs
    a few more batches than the rest, cheaper than the two extra launches of the chunked
    pre-aggregation.  Large snapshots scale it with the chunk size (many tiles per CU hide
    the spread)."""
    if num_edges > 65536:
        return int(max(64, 4 * chunk_edges))
    return int(min(256, max(64, max_deg)))


def _pack_tiles(inline_deg, budget):
    """Greedy tiles over the in-degree-sorted positive rows: up to 16 rows per tile while
    the tile's inline edges stay within `budget` (a row over budget contributes 0).
    Returns int32[n][2] = {start, count}."""
    n = len(inline_deg)
    if n == 0:
        return np.zeros((0, 2), np.int32)
    cs = np.concatenate([[0], np.cumsum(inline_deg, dtype=np.int64)])
    out = []
    a = 0
    while a < n:
        if cs[min(a + 16, n)] - cs[a] <= budget:  # the common case once past the hubs
            cnt = min(16, n - a)
        else:
            cnt = int(np.searchsorted(cs, cs[a] + budget, side="right")) - 1 - a
            cnt = max(1, min(16, cnt))
        out.append((a, cnt))
        a += cnt
    return np.asarray(out, dtype=np.int32).reshape(-1, 2)


def _chunk_spans(starts, lens, rows, chunk_edges):
    """Chunks {row, beg, end, slot} + fixups over explicit per-row CSR spans."""
    chunks_l, fix_l, nslot = [], [], 0
    for r, b, n in zip(rows, starts, lens):
        k = (int(n) + chunk_edges - 1) // chunk_edges
        if k == 1:
            chunks_l.append((r, b, b + n, -1))
            continue
        for i in range(k):
            chunks_l.append((r, b + i * chunk_edges, min(b + (i + 1) * chunk_edges, b + n), nslot + i))
        fix_l.append((r, nslot, nslot + k, 0))
        nslot += k
    fixups, nslot = group_fixups(fix_l, nslot)
    return np.array(chunks_l, dtype=np.int32).reshape(-1, 4), fixups, nslot


def _chunk_rows_spans(start, length, chunk_edges):
    """Chunk per-relation spans [start[r], start[r]+length[r]) of the r_to_e list."""
    R = len(start)
    order = np.arange(R)
    nz = length > 0
    rows, beg, lens = order[nz], start[nz], length[nz]
    ptr = np.zeros(len(rows) + 1, dtype=np.int64)
    # re-use _chunk_rows by building a synthetic pointer per relation
    chunks_l, fix_l, nslot = [], [], 0
    nchunk = (lens + chunk_edges - 1) // chunk_edges
    for r, b, n, k in zip(rows, beg, lens, nchunk):
        if k == 1:
            chunks_l.append((r, b, b + n, -1))
        else:
            for i in range(k):
                chunks_l.append((r, b + i * chunk_edges, min(b + (i + 1) * chunk_edges, b + n), nslot + i))
            fix_l.append((r, nslot, nslot + k, 0))
            nslot += k
    del ptr
    chunks = np.array(chunks_l, dtype=np.int32).reshape(-1, 4)
    fixups, nslot = group_fixups(fix_l, nslot)
    return chunks, fixups, nslot


# Relation means over entity blocks (hyperbolic_model.relation_context at large snapshots).  A
# relation's r_to_e list is ascending in entity id (np.unique), so cutting every forward
# relation's span at multiples of REL_BLOCK entity ids gives chunks that touch one block of x
# rows each.  The chunks of block k are dealt to the workgroups of XCD k % 8 (one wave per
# chunk, 4 waves per workgroup, workgroup w on XCD w % 8), in block order, so a block's rows come
# from HBM into that XCD's L2 once and serve every relation that lists them, instead of one HBM
# read per (relation, entity) pair.  Same kernel (regcn_segment_mean_f32), same values up to the
# fp32 association of each relation's partial sums (fixed order: deterministic).
REL_BLOCK = int(os.environ.get("REGCN_REL_BLOCK", "4096"))  # entity ids per block; 0: CSR chunks
REL_BLOCK_MIN_PAIRS = 1 << 20  # smaller snapshots keep the plain chunks (few rows, L2-resident)
REL_BLOCK_CHUNK = 256          # pairs per chunk inside one (relation, block) segment
_XCDS, _WAVES_PER_WG = 8, 4


# How blocked_span_chunks deals the block-ordered chunks to the XCD queues: "even" = xcds equal
# contiguous runs (a queue holds consecutive blocks; a block may straddle two queues), "mod" =
# block k to XCD k % xcds (a Zipf-hot source block makes its XCD's queue the longest)
XCD_DEAL = os.environ.get("REGCN_XCD_DEAL", "cost")
XCD_RUN_COST = int(os.environ.get("REGCN_XCD_RUN_COST", "7"))  # ~ L2 lines of a gathered row / an index


def blocked_span_chunks(span_rows, span_beg, span_len, keys, block, chunk, xcds=_XCDS, waves=_WAVES_PER_WG):
    """Chunks {row, beg, end, slot} and fix-ups over spans [span_beg[i], span_beg[i] +
    span_len[i]) of a position array whose `keys` (entity ids, ascending inside each span) pick
    the block key // block; a span is cut at block boundaries and every `chunk` positions.  A
    span's chunks get consecutive partial slots (none if it has one chunk: the wave finishes
    the row).  Dispatch order: position p belongs to XCD (p // waves) % xcds and XCD x takes the
    chunks of blocks x, x + xcds, ... in block order; padding chunks are empty spans into the
    spare last slot, which no fix-up reads.  torch tensors (any device) in, (chunks int32
    [n, 4], fixups int32 numpy [m, 4] after group_fixups, n_slots incl. the spare) out."""
    dev = span_len.device
    span_len = span_len.long()
    n = int(span_len.numel())
    total = int(span_len.sum()) if n else 0
    if total == 0:
        return torch.zeros(0, 4, dtype=torch.int32, device=dev), np.zeros((0, 4), np.int32), 0
    span_of = torch.repeat_interleave(torch.arange(n, device=dev), span_len)
    first = torch.cumsum(span_len, 0) - span_len
    pos = torch.arange(total, device=dev) + torch.repeat_interleave(span_beg.long() - first, span_len)
    blk = keys[pos].long() // block
    new_seg = torch.ones(total, dtype=torch.bool, device=dev)
    new_seg[1:] = (span_of[1:] != span_of[:-1]) | (blk[1:] != blk[:-1])
    seg_start = torch.nonzero(new_seg).squeeze(1)
    off = torch.arange(total, device=dev) - seg_start[torch.cumsum(new_seg, 0) - 1]
    cs = torch.nonzero(new_seg | (off % chunk == 0)).squeeze(1)
    ce = torch.cat([cs[1:], torch.tensor([total], device=dev)])
    c_span, c_blk = span_of[cs], blk[cs]
    n_per = torch.bincount(c_span, minlength=n)
    multi = n_per[c_span] > 1
    slot = torch.full_like(cs, -1)
    nslot = int(multi.sum())
    slot[multi] = torch.arange(nslot, device=dev)
    mr = torch.nonzero(n_per > 1).squeeze(1)
    s_first = torch.cumsum(n_per[mr], 0) - n_per[mr]
    fix = torch.stack([span_rows.long()[mr], s_first, s_first + n_per[mr], torch.zeros_like(mr)], 1).cpu().numpy()
    fixups, nslot = group_fixups(fix, nslot)
    chunks = torch.stack([span_rows.long()[c_span], pos[cs], pos[ce - 1] + 1, slot], 1)
    order = torch.sort(c_blk, stable=True).indices
    if XCD_DEAL == "even":  # the block-ordered chunks cut into xcds equal contiguous runs
        xq = torch.arange(order.numel(), device=dev) * xcds // max(order.numel(), 1)
    elif XCD_DEAL == "cost":  # ... with equal work per run: positions + XCD_RUN_COST per key run
        kv = keys[pos].long()
        head = new_seg.clone()
        head[1:] |= kv[1:] != kv[:-1]
        hc = torch.cat([torch.zeros(1, dtype=torch.long, device=dev), torch.cumsum(head.long(), 0)])
        first = torch.zeros(total, dtype=torch.bool, device=dev)
        first[cs] = True  # a chunk's first position starts a run in that chunk
        hc2 = torch.cat([torch.zeros(1, dtype=torch.long, device=dev), torch.cumsum((head | first).long(), 0)])
        runs = hc2[ce] - hc2[cs]
        del hc
        w = ((ce - cs) + XCD_RUN_COST * runs)[order]
        mid = torch.cumsum(w, 0) - w // 2
        xq = torch.clamp(mid * xcds // max(int(w.sum()), 1), max=xcds - 1)
    else:  # whole blocks round-robin
        xq = c_blk[order] % xcds
    queues = [order[xq == x] for x in range(xcds)]
    L = max(int(q.numel()) for q in queues)
    L = (L + waves - 1) // waves * waves
    out = torch.tensor([0, 0, 0, nslot], dtype=torch.long, device=dev).repeat(xcds * L, 1)
    q = torch.arange(L, device=dev)
    for x, qu in enumerate(queues):
        p = ((q // waves) * xcds + x) * waves + q % waves
        out[p[:qu.numel()]] = chunks[qu]
    return out.to(torch.int32), np.asarray(fixups, dtype=np.int32).reshape(-1, 4), nslot + 1


def spread_block(num_keys, block, xcds=_XCDS, per_xcd=2):
    """The block size blocked_span_chunks uses over `num_keys` key ids: `block`, shrunk so the
    key range holds at least per_xcd * xcds blocks (otherwise a small key range lands every
    chunk in a few XCD queues and pads the others with empty chunks)."""
    return max(64, min(int(block), -(-int(num_keys) // (per_xcd * xcds))))


def rel_block_lists(rel_idx, rel_start, rel_len, block, chunk=REL_BLOCK_CHUNK):
    """blocked_span_chunks over the forward relations' r_to_e spans (numpy in and out)."""
    rel_len = np.asarray(rel_len, dtype=np.int64)
    ch, fx, ns = blocked_span_chunks(torch.arange(len(rel_len)), torch.as_tensor(np.asarray(rel_start, np.int64)),
                                     torch.from_numpy(rel_len), torch.as_tensor(np.asarray(rel_idx, np.int64)),
                                     block, chunk)
    return ch.numpy(), fx, ns


def rel_block_work(g, R):
    """Device (chunks, fixups, n_slots) of rel_block_lists for snapshot `g` with R forward
    relations, built on first use
    and cached (None: the snapshot keeps the plain relation chunks)."""
    hit = g.__dict__.get("_rel_block")
    if hit is not None:
        return hit[0]
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        # built with host round trips, so not inside a HIP-graph capture: the plain chunks, and
        # cached, so later eager runs sum in the same order as the captured graph
        g.__dict__["_rel_block"] = (None,)
        return None
    wk = g.work()
    res = None
    if REL_BLOCK > 0 and int(wk["rel_idx"].numel()) // 2 >= REL_BLOCK_MIN_PAIRS:
        dev = wk["rel_idx"].device
        ch, fx, ns = blocked_span_chunks(torch.arange(R, device=dev), wk["rel_start"][:R], wk["rel_count"][:R].long(),
                                         wk["rel_idx"], spread_block(g.number_of_nodes(), REL_BLOCK), REL_BLOCK_CHUNK)
        res = (ch, torch.from_numpy(fx).to(dev), ns)
        from . import _lib
        _lib.publish()
    g.__dict__["_rel_block"] = (res,)
    return res


# The union hub pass over source blocks (hyperbolic_layers._heavy_aggregate, source runs): a
# hub row's edges in row/source order (row_src_cols) are ascending in source id, so the same
# cut at source-block boundaries, dealt to XCDs by block, lets the hub rows that list a source
# share its row from one L2.
HUB_BLOCK = int(os.environ.get("REGCN_HUB_BLOCK", "16384"))  # source ids per block; 0: plain chunks
HUB_BLOCK_MIN_EDGES = 1 << 20
HUB_CHUNK = int(os.environ.get("REGCN_HUB_CHUNK", "0"))  # edges per hub chunk; 0: hub_chunk()
HUB_CHUNKS_MIN = 16384


def hub_chunk(total_edges, chunk_edges):
    """Edges per hub-pass chunk (one wave each): the snapshot's chunk size, shrunk (not below
    256) so the pass has at least HUB_CHUNKS_MIN chunks.  An owner-partitioned rank holds ~1/8
    of the hub edges: config 5's 8-rank simulation at 1024 / 256 edges per chunk runs 5.42 /
    5.21 ms of encoder per rank (profiles/r4_hub_chunk_sweep.txt).  The whole config-5 snapshot
    keeps 1024: its hub rows hold ~32.7M of the 50M directed edges, ceil(32.7M / 16384) = 1,996
    > 1024 (a rank's ~4.1M give 250 -> the 256 floor)."""
    if HUB_CHUNK:
        return max(HUB_CHUNK, 64)
    base = max(int(chunk_edges or 1024), 64)
    return min(base, max(256, -(-int(total_edges) // HUB_CHUNKS_MIN)))


def hub_block_work(g):
    """Device (chunks, fixups, n_slots) of the hub rows' edge spans cut at source blocks
    (blocked_span_chunks over row_src_cols), built on first use and cached; None keeps the
    plain heavy chunks."""
    hit = g.__dict__.get("_hub_block")
    if hit is not None:
        return hit[0]
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        g.__dict__["_hub_block"] = (None,)  # as rel_block_work: plain chunks, cached
        return None
    res = None
    wk = g.work()
    hc = wk["heavy_chunks"]
    if HUB_BLOCK > 0 and g.n_heavy and hc.numel():
        rows = wk["rows"][:g.n_heavy].long()
        beg = wk["rowptr"].long()[rows]
        ln = wk["rowptr"].long()[rows + 1] - beg
        total = int(ln.sum())
        if total >= HUB_BLOCK_MIN_EDGES:
            ss = g.row_src_cols()
            ch, fx, ns = blocked_span_chunks(rows, beg, ln, ss, spread_block(g.number_of_nodes(), HUB_BLOCK),
                                             hub_chunk(total, getattr(g, "chunk_edges", None)))
            res = (ch, torch.from_numpy(fx).to(ss.device), ns)
            from . import _lib
            _lib.publish()
    g.__dict__["_hub_block"] = (res,)
    return res


class DeviceSnapshotGraph(SnapshotGraph):
    """A SnapshotGraph whose CSR, r2e lists and work lists were built by the HIP kernels
    (csrc/graphbuild.hip) from the triples in HBM.  The device lists are bit-identical to
    the host build's; the host-side views (edges(), in_degrees(), r_to_e, `_host`) are
    copied back lazily, only when something asks for them."""

    def _lazy(self, key, fn):
        v = self.__dict__.get(key)
        if v is None:
            v = fn()
            self.__dict__[key] = v
        return v

    def _tri(self):
        return self._lazy("_tri_np", lambda: self._tri_dev.cpu().numpy())

    @property
    def src_np(self):
        t = self._tri()
        return self._lazy("_src", lambda: np.concatenate((t[:, 0], t[:, 2])))

    @property
    def dst_np(self):
        t = self._tri()
        return self._lazy("_dst", lambda: np.concatenate((t[:, 2], t[:, 0])))

    @property
    def type_np(self):
        t = self._tri()
        return self._lazy("_type", lambda: np.concatenate((t[:, 1], t[:, 1] + self.num_rels)))

    @property
    def in_deg_np(self):
        return self._lazy("_in_deg", lambda: self.dev_all["in_deg"].cpu().numpy().astype(np.int64))

    @property
    def r_to_e(self):
        return self._lazy("_r_to_e", lambda: torch.from_numpy(self.dev_all["rel_idx"].cpu().numpy().astype(np.int64)))

    @property
    def _host(self):
        return self._lazy("_host_cache", lambda: {k: v.cpu().numpy() for k, v in self.dev_all.items()
                                                  if k != "in_deg"})

    def in_degrees(self, v=None):
        deg = self.dev_all["in_deg"].long()
        if v is None:
            return deg
        idx = torch.as_tensor(list(v) if isinstance(v, range) else v, dtype=torch.long, device=deg.device)
        return deg[idx]

    def edges(self):
        return torch.from_numpy(self.src_np), torch.from_numpy(self.dst_np)

    def number_of_edges(self):
        return 2 * int(self._tri_dev.shape[0])

    def to(self, device):
        if isinstance(device, int):
            device = torch.device("cuda", device) if device >= 0 else torch.device("cpu")
        device = torch.device(device)
        if device == self.device:
            return self
        # another device: rebuild from the host view (rare: the graph is built where it is used)
        host = SnapshotGraph(self.num_nodes_, self.num_rels, self.src_np, self.dst_np, self.type_np, self.uniq_r,
                             self.r_len, self.r_to_e.tolist(), chunk_edges=self.chunk_edges, tile_budget=self.budget)
        return host.to(device)


def _ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


def build_sub_graph_device(num_nodes, num_rels, triples, device, chunk_edges=DEFAULT_CHUNK_EDGES, tile_budget=None):
    """rgcn/utils.py:100-134 on the device: two library calls
    (regcn_snapshot_csr_i32, regcn_snapshot_work_i32) with one small host read of the
    counts between them (the tile budget depends on the maximum in-degree) and one after
    (list lengths).  Returns a DeviceSnapshotGraph on `device`."""
    from . import _lib
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError("the device graph build needs a HIP device (got %s)" % device)
    V, R = int(num_nodes), int(num_rels)
    if isinstance(triples, torch.Tensor):
        tri = triples.to(device=device, dtype=torch.int64).reshape(-1, 3).contiguous()
        tri_np = None
    else:
        tri_np = np.ascontiguousarray(np.asarray(triples, dtype=np.int64).reshape(-1, 3))
        tri = torch.from_numpy(tri_np).to(device)
    T = int(tri.shape[0])
    E = 2 * T
    ce = int(chunk_edges) if chunk_edges else chunk_size_for(E)
    lib = _lib.lib()
    S = _lib.SNAP

    def i32(n):
        return torch.empty(max(int(n), 1), dtype=torch.int32, device=device)

    def cap(what):
        c = int(lib.regcn_snapshot_capacity(_lib.CAP[what], T, V, R, ce))
        if c < 0:
            raise RuntimeError("regcn_snapshot_capacity(%s) failed" % what)
        return c

    ws = torch.empty(int(lib.regcn_snapshot_workspace_bytes(T, V, R)), dtype=torch.uint8, device=device)
    stats = torch.zeros(S["NSTATS"], dtype=torch.int32, device=device)
    out = {
        "in_deg": i32(V), "rowptr": i32(V + 1), "col_src": i32(E), "col_type": i32(E),
        "norm": torch.empty(V, dtype=torch.float32, device=device),
        "rel_ent_count": i32(R), "rel_idx": i32(cap("REL_IDX")), "rel_start": i32(2 * R),
        "rel_count": torch.empty(2 * R, dtype=torch.float32, device=device),
    }
    etype = torch.empty(max(E, 1), dtype=torch.int64, device=device)
    enorm = torch.empty(max(E, 1), dtype=torch.float32, device=device)
    d = _lib.SnapshotDesc()
    d.triples = _ptr(tri) if T else None
    d.T, d.V, d.R, d.chunk_edges = T, V, R, ce
    d.workspace, d.ws_bytes, d.stats = _ptr(ws), ws.numel(), _ptr(stats)
    for k, v in out.items():
        setattr(d, k, _ptr(v))
    d.edge_type, d.edge_norm = _ptr(etype), _ptr(enorm)
    _lib.call_desc("regcn_snapshot_csr_i32", d)
    st = stats.cpu().numpy()
    if st[S["INVALID"]]:
        raise ValueError("%d triples hold an entity id outside [0, %d) or a relation id outside [0, %d)"
                         % (int(st[S["INVALID"]]), V, R))
    budget = int(tile_budget) if tile_budget else tile_budget_for(E, ce, int(st[S["MAX_DEG"]]))
    pack = min(32, budget) if E <= 65536 else budget
    work = {
        "rows": i32(V), "tiles": i32(2 * cap("TILES")), "item_ptr": i32(V + 1), "item_src": i32(cap("ITEMS")),
        "item_tl": i32(cap("ITEMS")), "chunks": i32(4 * cap("CHUNKS")), "fixups": i32(4 * cap("FIXUPS")),
        "heavy_chunks": i32(4 * cap("HEAVY_CHUNKS")), "heavy_fixups": i32(4 * cap("HEAVY_FIXUPS")),
        "rel_chunks": i32(4 * cap("REL_CHUNKS")), "rel_fixups": i32(4 * cap("REL_FIXUPS")),
    }
    d.budget, d.pack_items = budget, pack
    for k, v in work.items():
        setattr(d, k, _ptr(v))
    _lib.call_desc("regcn_snapshot_work_i32", d)
    st = stats.cpu().numpy().astype(np.int64)

    def rec(t, n, w):
        return t[:n * w].view(n, w)

    n_tiles = int(st[S["N_TILES"]])
    ch, hc, rc = S["CHUNKS"], S["HEAVY_CHUNKS"], S["REL_CHUNKS"]
    n_pairs = int(st[S["N_PAIRS"]])
    dev = {
        "col_src": out["col_src"][:E], "col_type": out["col_type"][:E],
        "chunks": rec(work["chunks"], st[ch], 4), "fixups": rec(work["fixups"], st[ch + 1], 4),
        "norm": out["norm"], "rel_idx": out["rel_idx"][:2 * n_pairs], "rel_count": out["rel_count"],
        "rel_chunks": rec(work["rel_chunks"], st[rc], 4), "rel_fixups": rec(work["rel_fixups"], st[rc + 1], 4),
        "rel_start": out["rel_start"], "rowptr": out["rowptr"], "rows": work["rows"][:V],
        "tiles": rec(work["tiles"], n_tiles, 2), "heavy_chunks": rec(work["heavy_chunks"], st[hc], 4),
        "heavy_fixups": rec(work["heavy_fixups"], st[hc + 1], 4), "item_src": work["item_src"][:st[S["N_ITEMS"]]],
        "item_tl": work["item_tl"][:st[S["N_ITEMS"]]], "item_ptr": work["item_ptr"][:n_tiles + 1],
    }
    g = object.__new__(DeviceSnapshotGraph)
    g.num_nodes_, g.num_rels, g.device = V, R, device
    g._tri_dev = tri
    if tri_np is not None:
        g._tri_np = tri_np
    cnt = out["rel_ent_count"][:R].cpu().numpy().astype(np.int64)
    present = np.nonzero(cnt)[0]
    g.uniq_r = np.concatenate((present, present + R))
    starts = np.cumsum(cnt[present]) - cnt[present]
    g.r_len = [(int(a), int(a + n)) for a, n in zip(starts, cnt[present])] + \
              [(int(n_pairs + a), int(n_pairs + a + n)) for a, n in zip(starts, cnt[present])]
    g.ndata = _Frame(id=torch.arange(V, dtype=torch.long, device=device).view(-1, 1), norm=out["norm"].view(-1, 1))
    g.edata = _Frame(type=etype[:E], norm=enorm[:E].view(-1, 1))
    g.chunk_edges, g.budget, g.pack_items = ce, budget, pack
    g.n_pos, g.n_pos_tiles = int(st[S["N_POS"]]), n_tiles
    g.n_heavy, g.heavy_slots = int(st[S["N_HEAVY"]]), int(st[hc + 2])
    g.n_slots, g.rel_slots = int(st[ch + 2]), int(st[rc + 2])
    g.rel_max_span = int(st[S["REL_MAX"]])
    g.dev = dev
    g.dev_all = dict(dev, in_deg=out["in_deg"][:V])
    return g


def build_sub_graph(num_nodes, num_rels, triples, use_cuda=False, gpu=0, chunk_edges=DEFAULT_CHUNK_EDGES,
                    tile_budget=None, device_build=True):
    """rgcn/utils.py:100-134 (same signature; returns a SnapshotGraph).  chunk_edges /
    tile_budget override the work-list heuristics (tests use them to force split rows).
    With use_cuda the snapshot is built on the device (build_sub_graph_device; its lists
    equal the host build's bit for bit); device_build=False keeps the numpy build."""
    if use_cuda and device_build:
        dev = torch.device("cuda", gpu) if isinstance(gpu, int) else torch.device(gpu)
        return build_sub_graph_device(num_nodes, num_rels, triples, dev, chunk_edges=chunk_edges,
                                      tile_budget=tile_budget)
    triples = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    s, r, o = triples[:, 0], triples[:, 1], triples[:, 2]
    src = np.concatenate((s, o))
    dst = np.concatenate((o, s))
    etype = np.concatenate((r, r + num_rels))
    uniq_r, r_len, r_to_e = r2e(triples, num_rels)
    g = SnapshotGraph(num_nodes, num_rels, src, dst, etype, uniq_r, r_len, r_to_e, chunk_edges=chunk_edges,
                      tile_budget=tile_budget)
    if use_cuda:
        g = g.to(gpu)
        g.r_to_e = torch.from_numpy(np.array(r_to_e, dtype=np.int64))  # :133
    return g
