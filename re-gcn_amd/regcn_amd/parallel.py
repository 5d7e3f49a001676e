"""Multi-GPU partitions of one snapshot, one process per GPU, RCCL.

Two partitionings of a message-passing layer over `world` ranks:

* ``"edge"`` — the north star's literal scheme: rank k aggregates the k-th contiguous slice
  of the destination-sorted edge list (balanced by edge count) into raw per-row partial
  sums (union: sum_e w_e (x_src + rel); Lorentz: the summed Lorentz points plus their
  time coordinate); one ``all_reduce(SUM)`` of the V x (d + 1) partials; every rank
  finishes the rows (norm / centroid -> log0) and runs the MFMA tail on all rows.
* ``"owner"`` — rank k owns a set of destination nodes (OwnerLayout: `chunks` groups of
  contiguous ids per rank, chunk-major so that chunk j of every rank is one contiguous id
  range) and runs the fused layer kernel on them only (gather + GEMMs + epilogue,
  rank-local).  The next layer reads only the tangent rows x = log0 h and the radii |h| of
  its rows' in-edge sources, so after each chunk's launch ONE ``all_to_all`` sends every rank
  exactly those rows (ExchangePlan; records of 816 B), on a side stream while the next chunk
  computes (without a known consumer: in-place ``all_gather`` of every row); the Poincare rows h
  stay rank-local (the decoder fetches the rows it needs, `fetch_rows`, and scores each
  rank's own rows as its candidates, CandidateShard).  The relation-context means are
  partitioned the same way (per-rank partial sums over owned entities, one all_reduce of
  R x d).  Which node goes to which rank is a relabelling of the entity ids
  (`EntityRelabel.balanced`): LPT on the per-entity in-degrees, so the ranks carry equal
  edge loads under power-law skew (partitioning 2).

`ShardedGraph` wraps a `SnapshotGraph` with one of the two; the HIP layers dispatch on it,
so `HyperbolicRecurrentRGCN.forward(g_list=[ShardedGraph, ...])` runs sharded.  The
collective helpers (`allreduce_partials`, `allgather_rows`) and the plans are plain
torch.distributed / numpy, covered on CPU with gloo (tests/test_parallel.py); the compute
between them is the HIP library (tests/test_gpu_parity.py simulates the ranks on one GPU).
"""
import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .graph import fused_work, group_fixups


def even_bounds(n, world):
    return [n * k // world for k in range(world + 1)]


# ------------------------------------------------------------------------------ plans
class EdgePlan:
    """Rank `rank`'s slice [e0, e1) of the destination-sorted edges: every chunk writes a
    raw partial slot; `fixups` sum each touched row's slots into the V-row partial buffer;
    `finish` = {row, row, row + 1} for every row with in-degree > 0 (identical on all ranks)."""

    def __init__(self, g, rank, world):
        rowptr = g.work()["rowptr"].cpu().numpy().astype(np.int64) if g.dev is not None \
            else g._host["rowptr"].astype(np.int64)
        V = g.number_of_nodes()
        E = int(rowptr[-1])
        self.e0, self.e1 = even_bounds(E, world)[rank:rank + 2]
        ce = g.chunk_edges
        # the rows the slice touches, cut into chunks of <= ce edges (vectorised: ~1M rows
        # at config 5), slots numbered in chunk order, one fix-up per touched row
        rows = np.nonzero((rowptr[:-1] < self.e1) & (rowptr[1:] > self.e0))[0]
        beg = np.maximum(rowptr[rows], self.e0)
        end = np.minimum(rowptr[rows + 1], self.e1)
        k = (end - beg + ce - 1) // ce
        first = np.cumsum(k) - k
        total = int(k.sum())
        i = np.arange(total, dtype=np.int64) - np.repeat(first, k)
        c_beg = np.repeat(beg, k) + i * ce
        c_end = np.minimum(c_beg + ce, np.repeat(end, k))
        self.chunks = np.stack([np.repeat(rows, k), c_beg, c_end, np.arange(total)], 1).astype(np.int32).reshape(-1, 4)
        fix = np.stack([rows, first, first + k, np.zeros_like(k)], 1).astype(np.int32).reshape(-1, 4)
        self.fixups, self.n_slots = group_fixups(fix, total)
        pos = np.nonzero(np.diff(rowptr) > 0)[0]
        self.finish = np.stack([pos, pos, pos + 1, np.zeros_like(pos)], 1).astype(np.int32).reshape(-1, 4)
        self.V = V

    def to(self, device):
        self.dev = {k: torch.from_numpy(getattr(self, k)).to(device) for k in ("chunks", "fixups", "finish")}
        return self


def owner_bounds(V, world):
    """Equal contiguous node blocks (all_gather needs equal slices); the last is short."""
    per = (V + world - 1) // world
    return per, [min(V, per * k) for k in range(world + 1)]


def owner_chunks(V, world):
    """Pipeline chunks per rank of the owner partition (auto): 4 from 64k rows per rank.  The
    8-rank config-5 simulation (bench owner_simulation, round 4; the hub pass and the gather
    over all of a rank's rows, only the tails per chunk; the sparse exchange): 9.26 / 9.45 ms
    per step predicted at 4 / 2 chunks (profiles/r4_owner_sim_sparse.txt)."""
    return 4 if world > 1 and -(-V // world) >= 65536 else 1


class OwnerLayout:
    """Node ids of the owner partition: [0, Vp) in chunks x world groups of cr ids; group
    g = j * world + k, ids [g cr, (g + 1) cr) clipped to V, is rank k's pipeline chunk j.
    Chunk j of all ranks is the contiguous range [j world cr, (j + 1) world cr), so its
    all_gather lands in place (no pack / unpack).  One chunk: rank k owns [k cr, (k + 1) cr).
    Arrays exchanged this way are Vp rows long (rows >= V are padding nobody reads)."""

    def __init__(self, V, world, chunks=1):
        self.V, self.world, self.chunks = int(V), int(world), int(chunks)
        self.cr = max(1, -(-self.V // (self.world * self.chunks)))
        self.Vp = self.cr * self.world * self.chunks

    def group(self, rank, j):
        a = (j * self.world + rank) * self.cr
        return min(a, self.V), min(a + self.cr, self.V)

    def ranges(self, rank):
        return [self.group(rank, j) for j in range(self.chunks)]

    def owner(self, ids):
        return (ids // self.cr) % self.world

    def sizes(self):
        """Rows per group, g = j * world + k."""
        return [self.group(g % self.world, g // self.world) for g in range(self.world * self.chunks)]


class OwnerView:
    """A rank's view of a snapshot under the owner partition: the global CSR and relation
    spans, and the fused-kernel work lists of the node ids [lo, hi) only (one pipeline
    chunk of the rank's rows, see ShardedGraph)."""

    def __init__(self, g, lo, hi, ranges=None):
        """Node ids [lo, hi), or the union of `ranges` (a rank's pipeline chunks: one gather
        launch over all of them, ShardedGraph.run_layer)."""
        self.g = g
        ranges = [(int(lo), int(hi))] if ranges is None else [(int(a), int(b)) for a, b in ranges]
        self.v0, self.v1 = ranges[0][0], ranges[-1][1]
        nodes = np.concatenate([np.arange(a, b) for a, b in ranges]) if ranges else np.zeros(0, np.int64)
        h = g._host
        fw = fused_work(nodes, g.in_deg_np, h["rowptr"].astype(np.int64),
                        h["col_src"].astype(np.int64), h["col_type"].astype(np.int64), g.budget, g.pack_items,
                        g.chunk_edges)
        self.fw = fw
        self.budget, self.n_pos, self.n_pos_tiles = g.budget, fw.n_pos, fw.n_pos_tiles
        self.n_heavy, self.heavy_slots = fw.n_heavy, fw.heavy_slots
        self._dev = None

    def row_type_cols(self):
        return self.g.row_type_cols()

    def row_src_cols(self):
        return self.g.row_src_cols()

    def number_of_nodes(self):  # the key range of the source-blocked hub lists: every node
        return self.g.number_of_nodes()

    def work(self):
        if self._dev is None:
            wk = dict(self.g.work())
            dev = wk["rowptr"].device
            wk.update({k: torch.from_numpy(v).to(dev) for k, v in self.fw.host.items()})
            self._dev = wk
        return self._dev

    def item_type_cols(self):
        """The view's inline items with each row's items in relation-type order (the crel
        gather's lists, regcn_snapshot_item_type_order_i32 over the view's tiles), cached."""
        t = self.__dict__.get("_item_type")
        if t is None:
            t = self.__dict__["_item_type"] = type_ordered_items(self.work(), self.n_pos_tiles,
                                                                self.g.number_of_nodes(), 2 * self.g.num_rels)
        return t


def type_ordered_items(wk, n_tiles, V, R2):
    """(item_src, item_tl) of work lists `wk` with each row's items in relation-type order."""
    n_items = int(wk["item_src"].numel())
    if n_items == 0:
        return wk["item_src"], wk["item_tl"]
    dev = wk["item_src"].device
    ws = torch.empty(int(_lib.lib().regcn_item_src_order_workspace_bytes(n_items, V)), dtype=torch.uint8, device=dev)
    out = (torch.empty(n_items, dtype=torch.int32, device=dev), torch.empty(n_items, dtype=torch.int32, device=dev))
    _lib.call("regcn_snapshot_item_type_order_i32", V, R2, int(n_tiles), n_items, _lib.iptr(wk["tiles"]),
              _lib.iptr(wk["item_ptr"]), _lib.iptr(wk["item_src"]), _lib.iptr(wk["item_tl"]), _lib.iptr(out[0]),
              _lib.iptr(out[1]), ws.data_ptr(), ws.numel(), _lib.stream())
    _lib.publish()
    return out


class HaloView:
    """A rank's OwnerView read through its halo numbering: every source id in the view's work
    lists that another rank owns is replaced by the index of its row in the rank's halo (the
    rows after the Vp owned ids, where the sparse exchange's all_to_alls land the received x
    and |h| rows in place: no scatter on the receiving side).  Owned ids are unchanged.  The
    hub pass keeps the base view's chunk lists (cut at the ORIGINAL source blocks: `hub_owner`),
    rebased onto compacted, remapped copies of its hub rows' spans (`hub_cols`)."""

    def __init__(self, view, remap):
        self.v, self.remap = view, remap
        self.hub_owner = view
        self._work = None

    def __getattr__(self, name):
        return getattr(self.__dict__["v"], name)

    def work(self):
        if self._work is None:
            wk = dict(self.v.work())
            if wk["item_src"].numel():
                wk["item_src"] = self.remap[wk["item_src"].long()].to(torch.int32)
            self._work = wk
        return self._work

    def item_type_cols(self):
        """The base view's type-ordered items with the sources remapped (the crel gather)."""
        t = self.__dict__.get("_item_type")
        if t is None:
            src, tl = self.v.item_type_cols()
            if src.numel():
                src = self.remap[src.long()].to(torch.int32)
            t = self.__dict__["_item_type"] = (src, tl)
        return t

    def hub_cols(self, cs, ct, ss, hc):
        """The hub pass's columns for this view: only the spans of the hub rows that chunk list
        `hc` names (the rank's own hub rows, a fraction of the snapshot's edges), compacted --
        row/type order sources remapped to halo rows, their types, row/source order sources
        remapped (ss may be None) -- and `hc` with its positions rebased onto the compacted
        arrays.  Cached per chunk list; int64 temporaries are hub-edge sized, not E sized."""
        cache = self.__dict__.setdefault("_hub_cols", {})
        key = (hc.data_ptr(), ss is None)
        hit = cache.get(key)
        if hit is not None:
            return hit
        if not hc.numel():
            out = cache[key] = (cs[:0], ct[:0], None if ss is None else ss[:0], hc)
            return out
        rowptr = self.v.g.work()["rowptr"]
        rows = hc[:, 0].long()
        urows = torch.unique(rows)
        st = rowptr[urows].long()
        ln = rowptr[urows + 1].long() - st
        off = torch.cumsum(ln, 0) - ln
        n = int(ln.sum())
        pos = torch.repeat_interleave(st - off, ln) + torch.arange(n, device=st.device)  # global position of slot i
        cs_c = self.remap[cs[pos].long()].to(torch.int32)
        ct_c = ct[pos].contiguous()
        ss_c = None if ss is None else self.remap[ss[pos].long()].to(torch.int32)
        shift = (off - st)[torch.searchsorted(urows, rows)].to(torch.int32)
        hc2 = hc.clone()
        hc2[:, 1] += shift
        hc2[:, 2] += shift
        del pos
        _lib.publish()
        out = cache[key] = (cs_c, ct_c, ss_c, hc2)
        return out


# ------------------------------------------------------------------ sparse exchange
def exchange_keys(g, layout):
    """The (receiver, row) pairs of the owner partition's exchange for consumer snapshot `g`:
    rank m needs row s of another rank when s is the source of an in-edge of one of m's rows
    (the next layer reads x[s] and |h|[s] for its messages; its own rows it computed itself).
    Returns (m, s) int64 tensors sorted by (m, s), on the graph's device; cached on `g`."""
    key = (layout.world, layout.chunks, layout.cr)
    hit = g.__dict__.get("_xkeys")
    if hit is not None and hit[0] == key:
        return hit[1]
    if getattr(g, "dev", None) is not None:
        wk = g.work()
        rowptr, src = wk["rowptr"].long(), wk["col_src"].long()
    else:
        rowptr = torch.from_numpy(g._host["rowptr"].astype(np.int64))
        src = torch.from_numpy(g._host["col_src"].astype(np.int64))
    V = g.number_of_nodes()
    E = int(rowptr[-1])
    src = src[:E]
    dev = src.device
    dst_owner = torch.repeat_interleave(layout.owner(torch.arange(V, device=dev)), rowptr[1:] - rowptr[:-1])
    remote = layout.owner(src) != dst_owner
    pairs = torch.unique(dst_owner[remote] * layout.Vp + src[remote])  # sorted: by receiver, then row
    out = (pairs // layout.Vp, pairs % layout.Vp)
    g.__dict__["_xkeys"] = (key, out)
    return out


class ExchangePlan:
    """Rank `rank`'s part of the owner partition's exchange for one consumer snapshot, per
    pipeline chunk j: the ids of its own chunk-j rows that each other rank needs (grouped by
    receiver in rank order, ascending inside a group), the ids it receives (grouped by sender,
    ascending), and the split sizes of ONE all_to_all_single (x | |h| packed, 804 B per row at
    d = 200).  Every rank derives its lists from the same global snapshot (exchange_keys), so a
    sender's group for m and m's group from that sender hold the same ids in the same order.
    Config 5 at 8 ranks: a rank needs ~46 % of the other ranks' rows (Zipf sources), against
    all of them in the all-gather (a direct full-mesh exchange over xGMI)."""

    def __init__(self, g, layout, rank):
        m, s = exchange_keys(g, layout)
        W, cr = layout.world, layout.cr
        k = layout.owner(s)
        j = (s // cr) // W
        self.world, self.chunks = W, []
        for jj in range(layout.chunks):
            sm = (k == rank) & (j == jj)
            rm = (m == rank) & (j == jj)
            send, recv = s[sm], s[rm]
            self.chunks.append((send, torch.bincount(m[sm], minlength=W).tolist(),
                                recv, torch.bincount(k[rm], minlength=W).tolist()))
        # the halo: every received id, chunk by chunk (inside a chunk by sender, ascending) --
        # the order in which the all_to_alls deliver the rows into the rows after the owned ids
        self.halo = torch.cat([c[2] for c in self.chunks]) if self.chunks else s[:0]
        off = np.cumsum([0] + [int(c[2].numel()) for c in self.chunks])
        self.halo_off = [int(v) for v in off]

    def remap(self, V, base):
        """Global id -> the index a consumer reads it at: owned and unreceived ids unchanged,
        received id halo[i] -> base + i (int64, on the plan's device; cached per base)."""
        hit = self.__dict__.get("_remap")
        if hit is not None and hit[0] == base:
            return hit[1]
        m = torch.arange(V, device=self.halo.device, dtype=torch.int64)
        m[self.halo] = base + torch.arange(self.halo.numel(), device=self.halo.device, dtype=torch.int64)
        self.__dict__["_remap"] = (base, m)
        return m

    def rows_received(self):
        return sum(sum(c[3]) for c in self.chunks)

    def send_slots(self, j, lo, n):
        """Chunk j's send block as seen from its rows (the tail writes it, regcn_layer_desc
        send_*): (ptr, pos) int32 with row id lo + i going to block slots pos[ptr[i] .. ptr[i + 1])
        -- the positions of id lo + i in chunk j's send list (one per receiver that reads it).
        None when the chunk sends nothing or an id falls outside [lo, lo + n)."""
        cache = self.__dict__.setdefault("_send_slots", {})
        key = (j, lo, n)
        if key not in cache:
            send = self.chunks[j][0]
            out = None
            if send.numel() and int(send.min()) >= lo and int(send.max()) < lo + n:
                order = torch.argsort(send, stable=True)
                ptr = torch.zeros(n + 1, device=send.device, dtype=torch.int64)
                ptr[1:] = torch.cumsum(torch.bincount(send - lo, minlength=n), 0)
                out = (ptr.int(), order.int())
            cache[key] = out
        return cache[key]

    def send_block(self, j, lo, n, d):
        """(send descriptor for the chunk-j tail, (x block, |h| vector)) or None: fresh buffers
        of chunk j's send list the tail fills (see send_slots)."""
        sl = self.send_slots(j, lo, n)
        if sl is None:
            return None
        m = self.chunks[j][0].numel()
        dev = self.chunks[j][0].device
        xs = torch.empty(m, d, device=dev, dtype=torch.float32)
        r1 = torch.empty(m, device=dev, dtype=torch.float32)
        return (lo, n, sl[0], sl[1], xs, r1), (xs, r1)

    def link_rows(self, j):
        """The largest per-peer row count of chunk j's exchange, either direction (each peer
        pair has its own xGMI link, so the exchange takes max over links)."""
        _, ss, _, rs = self.chunks[j]
        return max(max(ss), max(rs)) if ss else 0


def pack_rows(xn, rn, ids):
    """(len(ids), d + 4) records [x row, |h|, pad] of rows `ids` (regcn_pack_rows_f32)."""
    d = xn.shape[1]
    out = torch.empty(ids.numel(), d + 4, device=xn.device, dtype=torch.float32)
    _lib.call("regcn_pack_rows_f32", _lib.fptr(xn, "x"), _lib.fptr(rn, "radius"), _lib.dptr(ids, torch.int64, "ids"),
              ids.numel(), d, _lib.fptr(out), _lib.stream())
    return out


def unpack_rows(buf, ids, xn, rn):
    """Records of pack_rows written back to rows `ids` of xn / rn (regcn_unpack_rows_f32)."""
    _lib.call("regcn_unpack_rows_f32", _lib.fptr(buf, "records"), _lib.dptr(ids, torch.int64, "ids"), ids.numel(),
              xn.shape[1], _lib.fptr(xn, "x"), _lib.fptr(rn, "radius"), _lib.stream())


def exchange_rows(chunk, xn, rn, group=None, pack=pack_rows, unpack=unpack_rows):
    """One chunk of an ExchangePlan: this rank's rows other ranks read (x | |h| records),
    ONE all_to_all_single, the received records written into xn / rn in place.  `pack` /
    `unpack`: the HIP kernels (a CPU test of the plan passes torch stand-ins)."""
    sidx, ss, ridx, rs = chunk
    send = pack(xn, rn, sidx)
    recv = torch.empty(ridx.numel(), send.shape[1], device=xn.device, dtype=xn.dtype)
    _all_to_all_into(recv, send, rs, ss, group)
    unpack(recv, ridx, xn, rn)


# The sparse exchange delivers into the receiver's halo rows (HaloView; two all_to_alls per
# chunk, x rows and |h|, no receive-side scatter); 0: one all_to_all of pack_rows' (d + 4)-float
# records scattered into the global rows by unpack_rows (round 4)
HALO = os.environ.get("REGCN_HALO", "1") != "0"
# The large-snapshot tails write the send block themselves (regcn_layer_desc send_*); 0: a gather
# kernel after each chunk's tail (regcn_gather_rows_f32)
SEND_FROM_TAIL = os.environ.get("REGCN_SEND_FROM_TAIL", "1") != "0"


def record_bytes(plan, d):
    """Bytes per exchanged row: x and |h|, (d + 1) floats (the in-place all-gathers, plan None,
    and the halo exchange); pack_rows' (d + 4)-float records without the halo."""
    return (d + 1) * 4 if (plan is None or HALO) else (d + 4) * 4


def exchange_halo(plan, j, xn, rn, base, group=None, gather=None):
    """Chunk j of an ExchangePlan through the halo: this rank's rows other ranks read gathered
    into a contiguous x block and |h| vector (regcn_gather_rows_f32), two all_to_all_singles
    landing the received rows at rows base + halo_off[j] .. of xn / rn (the consumer's HaloView
    numbering): no scatter.  `gather`: a stand-in for the HIP gather (CPU tests)."""
    sidx, ss, _, rs = plan.chunks[j]
    d = xn.shape[1]
    xs, r1 = (gather or gather_rows)(xn, rn, sidx)
    a, b = base + plan.halo_off[j], base + plan.halo_off[j + 1]
    _all_to_all_into(xn[a:b], xs, rs, ss, group)
    _all_to_all_into(rn[a:b], r1, rs, ss, group)
    return d


def gather_rows(xn, rn, ids):
    """(x rows, |h| values) of rows `ids`, contiguous (regcn_gather_rows_f32)."""
    d = xn.shape[1]
    xs = torch.empty(ids.numel(), d, device=xn.device, dtype=torch.float32)
    r1 = torch.empty(ids.numel(), device=xn.device, dtype=torch.float32)
    _lib.call("regcn_gather_rows_f32", _lib.fptr(xn, "x"), _lib.fptr(rn, "radius"), _lib.dptr(ids, torch.int64, "ids"),
              ids.numel(), d, _lib.fptr(xs), _lib.fptr(r1), _lib.stream())
    return xs, r1


FULL_EXCHANGE = "all rows"  # ShardedGraph.consumers: the next consumer is unknown -> all-gather


# ------------------------------------------------------------- balanced entity relabel
def _lpt(load, caps, head=None):
    """Group (0 .. len(caps) - 1) of every item: longest-processing-time first -- items by
    descending load, each to the least-loaded group with room (caps[g] items) -- for the
    `head` heaviest items; the light tail dealt round-robin, heaviest first, over the groups
    in ascending load order, each up to its room.  sum(caps) == len(load)."""
    import heapq
    load = np.asarray(load, dtype=np.float64)
    caps = np.asarray(caps, dtype=np.int64)
    n, G = len(load), len(caps)
    if int(caps.sum()) != n:
        raise ValueError("group capacities must sum to the item count")
    order = np.argsort(-load, kind="stable")
    out = np.empty(n, dtype=np.int64)
    cnt = np.zeros(G, dtype=np.int64)
    tot = np.zeros(G)
    K = min(n, head if head is not None else 4096 * G)
    heap = [(0.0, g) for g in range(G) if caps[g] > 0]
    heapq.heapify(heap)
    for i in order[:K]:
        lo, g = heapq.heappop(heap)
        out[i] = g
        cnt[g] += 1
        tot[g] = lo + load[i]
        if cnt[g] < caps[g]:
            heapq.heappush(heap, (tot[g], g))
    rest = order[K:]
    if len(rest):
        room = caps - cnt
        pos = np.empty(G, dtype=np.int64)
        pos[np.argsort(tot, kind="stable")] = np.arange(G)
        g_rep = np.repeat(np.arange(G), room)
        r_idx = np.arange(len(g_rep)) - np.repeat(np.cumsum(room) - room, room)
        out[rest] = g_rep[np.argsort(r_idx * G + pos[g_rep], kind="stable")]
    return out


class EntityRelabel:
    """A permutation of the entity ids (old id -> new id) that balances the owner partition:
    the model is equivariant under it (entity-indexed parameters permuted alike, the triples
    relabelled), so every MRR is unchanged while rank k's rows -- the ids OwnerLayout gives it
    -- carry ~1/world of the edges under power-law skew (a Zipf(1.1) hub holds ~9 % of a
    snapshot's edges; equal contiguous id blocks leave the hubs wherever the ids put them)."""

    # every entity-indexed parameter / buffer of the hyperbolic and Euclidean models: the
    # embedding table, the radii, the scorers' per-entity bias (RotH / MuRP / AttH `entity_bias`,
    # hyperbolic_decoder.py:166; ConvTransE's `b`, hyperbolic_decoder.py:568, rrgcn.py:71)
    ENTITY_TENSORS = ("dynamic_emb", "radius_static", "radius_target", "decoder_ob.entity_bias", "decoder_ob.b")

    def __init__(self, perm):
        self.perm = np.asarray(perm, dtype=np.int64)
        self.inv = np.empty_like(self.perm)
        self.inv[self.perm] = np.arange(len(self.perm))
        self._dev = {}

    @classmethod
    def balanced(cls, snapshots, V, world, chunks=None):
        """LPT over the entities' in-degrees in the doubled snapshot graphs (one per subject and
        object occurrence, rgcn/utils.py:116-118) summed over `snapshots` (triple arrays): first
        to ranks (equal row counts), then inside each rank to its pipeline chunks."""
        chunks = chunks or owner_chunks(V, world)
        lay = OwnerLayout(V, world, chunks)
        deg = np.zeros(V, dtype=np.float64)
        for tr in snapshots:
            tr = np.asarray(tr)
            deg += np.bincount(tr[:, 0], minlength=V) + np.bincount(tr[:, 2], minlength=V)
        size = np.array([hi - lo for lo, hi in lay.sizes()], dtype=np.int64)  # g = j * world + k
        rank_cap = size.reshape(chunks, world).sum(0)
        rank_of = _lpt(deg, rank_cap)
        perm = np.empty(V, dtype=np.int64)
        for k in range(world):
            mine = np.nonzero(rank_of == k)[0]
            caps = size.reshape(chunks, world)[:, k]
            chunk_of = _lpt(deg[mine], caps) if chunks > 1 else np.zeros(len(mine), np.int64)
            for j in range(chunks):
                rows = mine[chunk_of == j]  # ascending old ids
                lo, _ = lay.group(k, j)
                perm[rows] = lo + np.arange(len(rows))
        return cls(perm)

    def loads(self, snapshots, world, chunks=None):
        """Per-rank directed in-edges of each snapshot under this relabel ([n_snap][world])."""
        V = len(self.perm)
        lay = OwnerLayout(V, world, chunks or owner_chunks(V, world))
        out = []
        for tr in snapshots:
            tr = np.asarray(tr)
            own = lay.owner(self.perm[np.concatenate([tr[:, 0], tr[:, 2]])])
            out.append(np.bincount(own, minlength=world).tolist())
        return out

    def _t(self, which, device):
        key = (which, str(device))
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(getattr(self, which)).to(device)
        return self._dev[key]

    def triples(self, tr):
        """(s, r, o) rows with s and o relabelled (numpy or torch, a copy)."""
        if torch.is_tensor(tr):
            p = self._t("perm", tr.device)
            out = tr.clone()
            out[:, 0] = p[tr[:, 0].long()].to(tr.dtype)
            out[:, 2] = p[tr[:, 2].long()].to(tr.dtype)
            return out
        tr = np.asarray(tr)
        out = tr.copy()
        out[:, 0] = self.perm[tr[:, 0]]
        out[:, 2] = self.perm[tr[:, 2]]
        return out

    def model(self, m):
        """Permute the entity-indexed parameters / buffers of a model in place (new row
        perm[i] = old row i); in-place writes bump the version counters the caches key on."""
        names = dict(m.named_parameters())
        names.update(dict(m.named_buffers()))
        V = len(self.perm)
        with torch.no_grad():
            for n in self.ENTITY_TENSORS:
                t = names.get(n)
                if t is not None:
                    if t.shape[0] != V:
                        raise ValueError("%s has %d rows, the relabel %d entities" % (n, t.shape[0], V))
                    t.copy_(t[self._t("inv", t.device)])
        from .weights import invalidate
        invalidate(m)
        return m


# -------------------------------------------------------------------------- collectives
def allreduce_partials(P, group=None):
    """Sum the ranks' raw partial rows (edge partition)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(P, op=dist.ReduceOp.SUM, group=group)
    return P


def allgather_rows(full, per, group=None):
    """full: (world * per, ...) with this rank's block [rank*per, (rank+1)*per) filled;
    afterwards every block is filled on every rank (owner partition)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        rank = dist.get_rank(group)
        chunk = full[rank * per:(rank + 1) * per].clone()
        _all_gather_into(full, chunk, group)
    return full


def _all_gather_into(out, chunk, group=None):
    """all_gather_into_tensor; a gloo group (CPU tests, ranks sharing one GPU in the GPU
    tests) gathers through host tensors."""
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(chunk, device="cpu") for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, chunk.cpu(), group=group)
        out.copy_(torch.cat(parts).to(out.device))
    else:
        dist.all_gather_into_tensor(out, chunk, group=group)


def _all_to_all_into(out, inp, out_splits, in_splits, group=None):
    """all_to_all_single with split sizes (rows); gloo through host tensors."""
    if dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o.to(out.device))
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def allgather_fused(tensors, per, rows=None, group=None):
    """One collective for several row-aligned tensors (h, log0 h, |h| of the owner
    partition): this rank's rows `rows` (a slice of its block, default all `per`) of every
    tensor packed into one (n, W) buffer, ONE all_gather, unpacked into the same rows of
    every rank's block.  Each tensor is (world * per, ...) ."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return tensors
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    a, b = (0, per) if rows is None else (rows.start, rows.stop)
    flat = [t.view(world, per, -1) for t in tensors]
    send = torch.cat([f[rank, a:b] for f in flat], 1).contiguous()
    recv = torch.empty(world, b - a, send.shape[1], device=send.device, dtype=send.dtype)
    _all_gather_into(recv.view(world * (b - a), -1), send, group)
    off = 0
    for f in flat:
        w = f.shape[2]
        f[:, a:b].copy_(recv[:, :, off:off + w])
        off += w
    return tensors


# ---------------------------------------------------------------------- sharded layers
def owned_rel_spans(rel_idx, rel_count, ranges, Vp):
    """The forward relations' r_to_e spans (consecutive in rel_idx, relation r holding
    rel_count[r] entries, ascending entity ids) cut to the entity id ranges [lo, hi): span
    r * len(ranges) + q holds relation r's entities in range q.  Returns (rows, beg, len)
    tensors (span row = r * n_ranges + q) on rel_idx's device."""
    dev = rel_idx.device
    cnt = rel_count.long()
    R, nq = int(cnt.numel()), len(ranges)
    ids = rel_idx[:int(cnt.sum())].long()
    Vk = int(Vp) + 1  # key = relation * Vk + id ascends over the whole forward list
    key = torch.repeat_interleave(torch.arange(R, device=dev), cnt) * Vk + ids
    lo = torch.tensor([a for a, _ in ranges], device=dev, dtype=torch.long).repeat(R)
    hi = torch.tensor([b for _, b in ranges], device=dev, dtype=torch.long).repeat(R)
    rr = torch.arange(R, device=dev).repeat_interleave(nq)
    beg = torch.searchsorted(key, rr * Vk + lo)
    end = torch.searchsorted(key, rr * Vk + hi)
    return torch.arange(R * nq, device=dev), beg, end - beg


class ShardedGraph:
    """A SnapshotGraph partitioned across the ranks of `group` (see module docstring).
    Everything but the message-passing layers (relation spans, degrees, ...) is the
    wrapped graph's."""

    # owner partition: a rank's rows run in this many chunks, each one's rows all-gathered on a
    # side stream while the next chunk computes (auto: owner_chunks)
    pipeline_chunks = None

    def __init__(self, g, partition="owner", group=None, rank=None, world=None, chunks=None):
        if partition not in ("edge", "owner"):
            raise ValueError("partition must be 'edge' or 'owner'")
        self.g, self.partition, self.group = g, partition, group
        if rank is None:
            rank = dist.get_rank(group) if dist.is_initialized() else 0
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank, self.world = rank, world
        self.chunks = chunks
        self.plan = EdgePlan(g, rank, world).to(g.device) if partition == "edge" else None
        self.layout, self.views, self.rank_view = None, [], None
        if partition == "owner":
            V = g.number_of_nodes()
            k = chunks or self.pipeline_chunks or owner_chunks(V, world)
            self.layout = OwnerLayout(V, world, k)
            self.views = [((lo, hi), OwnerView(g, lo, hi)) for lo, hi in self.layout.ranges(rank)]
            # all of the rank's rows as one view: with the large-snapshot layer path the hub
            # pass and the gather run once over them, only the tails per chunk
            self.rank_view = OwnerView(g, 0, 0, ranges=self.layout.ranges(rank)) if len(self.views) > 1 else None
        self._comm = None
        self._rel = None
        # collectives only inside a process group of world > 1 (a single-process simulation of
        # one rank, bench.py's owner_simulation, runs the rank's launches alone)
        self.collective = dist.is_initialized() and dist.get_world_size(group) > 1
        self.exchanged_bytes = 0  # bytes this rank received in the owner exchanges (bench)
        # (after a non-step layer, after the step layer) the snapshot whose layer reads the new
        # rows next, set per timestep by HyperbolicRecurrentRGCN.forward: a ShardedGraph (the
        # sparse exchange of its ExchangePlan), None (nothing reads them: no exchange) or
        # FULL_EXCHANGE; unset (None): every layer all-gathers every row
        self.consumers = None

    def exchange_plan(self, step):
        """None: all-gather every row; False: no exchange; else the ExchangePlan of the layer's
        consumer (self for a cell's inner layer, the next timestep's snapshot after the step)."""
        if self.consumers is None:
            return None
        target = self.consumers[1] if step is not None else self.consumers[0]
        if target is None:
            return False
        if target is FULL_EXCHANGE:
            return None
        return target.plan_for(self.rank)

    def exchange_target(self, step):
        """The consumer object of this layer's rows (see exchange_plan), or None."""
        if self.consumers is None:
            return None
        t = self.consumers[1] if step is not None else self.consumers[0]
        return None if t is FULL_EXCHANGE else t

    def plan_for(self, rank):
        """Rank `rank`'s ExchangePlan with this snapshot as the consumer (cached)."""
        plans = self.__dict__.setdefault("_xplans", {})
        key = (rank, self.world, self.layout.chunks)
        if key not in plans:
            plans[key] = ExchangePlan(self.g, self.layout, rank)
        return plans[key]

    def halo_views(self, plan, base):
        """(the rank's whole-rows view, its chunk views) read through the halo numbering of
        `plan` (this snapshot as the consumer) with the halo at rows [base, base + H)."""
        cache = self.__dict__.setdefault("_halo_views", {})
        if base not in cache:
            remap = plan.remap(self.g.number_of_nodes(), base)
            rv = HaloView(self.rank_view, remap) if self.rank_view is not None else None
            cache[base] = (rv, [HaloView(v, remap) for _, v in self.views])
        return cache[base]

    def init_rows(self, k=None):
        """(own ids, halo ids), int32 on the device: the rows of the initial entity state rank k
        (default this rank) reads -- its own rows, and this snapshot's halo (the sources of its
        edges that other ranks own: all its first layer reads besides its own rows)."""
        k = self.rank if k is None else k
        cache = self.__dict__.setdefault("_init_rows", {})
        if k not in cache:
            dev = self.g.device
            own = [torch.arange(a, b, device=dev, dtype=torch.int32) for a, b in self.layout.ranges(k) if b > a]
            own = torch.cat(own) if own else torch.zeros(0, device=dev, dtype=torch.int32)
            cache[k] = (own, self.plan_for(k).halo.to(dev, torch.int32))
        return cache[k]

    def halo_initial_state(self):
        """Whether initial_state applies: the owner partition of > 1 ranks with the halo
        exchange (the first layer then reads its sources through the halo views)."""
        return self.partition == "owner" and self.world > 1 and HALO

    @staticmethod
    def _init_launch(dyn, r_static, src, dst, h, x, r, c, layer_norm):
        if src.numel():
            _lib.call("regcn_init_entity_rows_f32", _lib.fptr(dyn, "dynamic_emb"), _lib.fptr(r_static),
                      _lib.iptr(src), _lib.iptr(dst) if dst is not None else None, src.numel(), dyn.shape[1],
                      float(c), int(bool(layer_norm)), _lib.fptr(h) if h is not None else None, _lib.fptr(x),
                      _lib.fptr(r), _lib.stream())

    def initial_state(self, dyn, r_static, c, layer_norm):
        """The initial entity state (h, x = log0 h, |h|; regcn_init_entities_f32's map,
        hyperbolic_model.py:779-782) only where this rank reads it: its own rows at their ids and
        this snapshot's halo at rows Vp.. (x and |h|), x tagged for the halo views as a layer's
        output is, so the first layer reads its sources there.  Replaces every rank mapping all
        V rows (config 5 at 8 ranks: 0.6 ms per step on every rank).  Rows outside are unset."""
        lay = self.layout
        V, d = dyn.shape
        own, halo = self.init_rows()
        H = halo.numel()
        h = torch.empty(lay.Vp, d, device=dyn.device, dtype=torch.float32)
        x = torch.empty(lay.Vp + H, d, device=dyn.device, dtype=torch.float32)
        r = torch.empty(lay.Vp + H, device=dyn.device, dtype=torch.float32)
        self._init_launch(dyn, r_static, own, own, h, x, r, c, layer_norm)
        self._init_launch(dyn, r_static, halo, None, None, x[lay.Vp:], r[lay.Vp:], c, layer_norm)
        xv = x[:V]
        xv._regcn_halo = (self, x, r)
        return h[:V], xv, r[:V]

    def link_bytes(self, plan, j, d):
        """Bytes on the busiest peer link in chunk j's exchange (the all-gather: one chunk of
        rows from every peer)."""
        if plan is False:
            return 0
        rows = self.layout.cr if plan is None else plan.link_rows(j)
        return rows * record_bytes(plan, d)

    def __getattr__(self, name):  # delegate the DGL-visible surface and work lists
        return getattr(self.__dict__["g"], name)

    def work(self):
        return self.g.work()

    def to(self, device):
        device = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        if device == self.g.device:
            return self
        return ShardedGraph(self.g.to(device), self.partition, self.group, self.rank, self.world, self.chunks)

    def candidate_ranges(self, N):
        """The entity ids this rank scores as candidates: its own rows (owner partition: the
        rows whose Poincare embedding it computed), an even slice otherwise."""
        if self.partition == "owner" and self.layout.V == N:
            return [r for r in self.layout.ranges(self.rank) if r[1] > r[0]]
        b = even_bounds(N, self.world)
        return [(b[self.rank], b[self.rank + 1])]

    # ---- edge partition pieces (also used by the single-GPU rank simulation in tests)
    def edge_partials(self, mode, x, r, rel, w_rel, nb, gamma, c):
        """This rank's raw partial sums: (V, d + 4) with the Lorentz time coordinate at
        column d, zero for rows without edges in the slice."""
        wk = self.g.work()
        V, d = x.shape
        stride = d + 4
        pl = self.plan.dev
        S = torch.empty(max(self.plan.n_slots, 1), stride, device=x.device, dtype=torch.float32)
        P = torch.zeros(V, stride, device=x.device, dtype=torch.float32)
        f, i = _lib.fptr, _lib.iptr
        ch = pl["chunks"]
        if mode == _lib.AGG_LORENTZ:
            cs, ct = self.g.row_type_cols()
            _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(w_rel), i(cs), i(ct),
                      i(ch), ch.shape[0], None, 0, nb, float(c), d, f(S), stride, f(P), _lib.stream())
        elif mode == _lib.AGG_UNION:
            _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                      f(wk["norm"]), i(ch), ch.shape[0], None, 0, float(gamma), d, f(S), stride, f(P),
                      _lib.stream())
        else:
            _lib.call("regcn_euclid_aggregate_f32", f(x), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                      f(wk["norm"]), i(ch), ch.shape[0], None, 0, d, f(S), stride, f(P), _lib.stream())
        width = d + 1 if mode == _lib.AGG_LORENTZ else d
        fx = pl["fixups"]
        _lib.call("regcn_partial_sum_f32", f(S), stride, i(fx), fx.shape[0], width, f(P), stride, _lib.stream())
        return P

    def edge_finish(self, mode, P, x, r, rel, w_rel, nb, gamma, c):
        """Finished aggregation rows (norm scale, or Lorentz centroid -> log0) from the
        all-reduced partials."""
        wk = self.g.work()
        V, d = x.shape
        stride = P.shape[1]
        agg = torch.zeros(V, d, device=x.device, dtype=torch.float32)
        fn = self.plan.dev["finish"]
        f, i = _lib.fptr, _lib.iptr
        if mode == _lib.AGG_LORENTZ:
            _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(w_rel), i(wk["col_src"]), i(wk["col_type"]),
                      None, 0, i(fn), fn.shape[0], nb, float(c), d, f(P), stride, f(agg), _lib.stream())
        elif mode == _lib.AGG_UNION:
            _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                      f(wk["norm"]), None, 0, i(fn), fn.shape[0], float(gamma), d, f(P), stride, f(agg),
                      _lib.stream())
        else:
            _lib.call("regcn_euclid_aggregate_f32", f(x), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                      f(wk["norm"]), None, 0, i(fn), fn.shape[0], d, f(P), stride, f(agg), _lib.stream())
        return agg

    def _rank_launches(self, mode, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                       drop_mask, c, euclid, step, out, gate, exchange, views=None, send=None):
        """This rank's launches of one layer into `out`, exchange(j) after chunk j's rows are
        final.  Large snapshots: the hub pass and the gather once over all of the rank's rows,
        then each chunk's tail (full-size launches but the tails); otherwise each chunk's whole
        layer launch.  views: (whole-rows view, chunk views) to read x / r through (the halo
        views when the input came through the halo exchange; default the plain views).  send(j):
        chunk j's send-block descriptor for its tail (ExchangePlan.send_block) or None; only the
        large-snapshot tails take it (exchange(j) gathers the rows otherwise)."""
        from .hyperbolic_layers import _use_rowtail, run_layer, run_layer_chunked
        V, d = x.shape
        rv, cvs = views if views is not None else (self.rank_view, [v for _, v in self.views])
        if rv is not None and _use_rowtail(V, int(rv.fw.host["rows"].shape[0]), d, prev_t, drop_mask, False):
            run_layer_chunked(mode, rv, cvs, x, r, rel, w_rel, nb, gamma, w_n, w_loop,
                              w_evolve, c, euclid, step, out, gate, exchange, send=send)
            return
        for j, view in enumerate(cvs):
            run_layer(mode, view, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                      drop_mask, c, euclid=euclid, step=step, out=out, gate=gate)
            exchange(j)

    def run_layer(self, mode, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                  drop_mask, c, euclid=False, step=None, gate=None):
        """The sharded counterpart of hyperbolic_layers.run_layer (same arguments/returns)."""
        from .hyperbolic_layers import run_layer
        V, d = x.shape
        if self.partition == "edge":
            P = self.edge_partials(mode, x, r, rel, w_rel, nb, gamma, c)
            allreduce_partials(P, self.group)
            agg = self.edge_finish(mode, P, x, r, rel, w_rel, nb, gamma, c)
            return run_layer(_lib.AGG_NONE, self.g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t,
                             w_skip, b_skip, drop_mask, c, euclid=euclid, step=step, agg=agg)
        lay = self.layout
        W, cr = self.world, lay.cr
        # the input came through the halo exchange for this snapshot: read the full buffers
        # (owned rows + halo) through the halo views
        tag = getattr(x, "_regcn_halo", None)
        views, xin, rin = None, x, r
        if tag is not None and tag[0] is self:
            xin, rin = tag[1], tag[2]
            views = self.halo_views(self.plan_for(self.rank), lay.Vp)
        plan = self.exchange_plan(step) if W > 1 else False
        halo_out = HALO and isinstance(plan, ExchangePlan) and self.collective
        H = plan.halo.numel() if halo_out else 0
        h = torch.empty(lay.Vp, d, device=x.device, dtype=torch.float32)
        xn = torch.empty(lay.Vp + H, d, device=x.device, dtype=torch.float32)
        rn = torch.empty(lay.Vp + H, device=x.device, dtype=torch.float32)
        # the rank's rows in pipeline chunks: after chunk j's launch, chunk j of every rank --
        # one contiguous id range -- is all-gathered in place, x and |h| (804 B per row), on a
        # side stream while chunk j + 1 computes (partitioning 2 with overlap)
        cur = torch.cuda.current_stream(x.device) if x.is_cuda else None
        comm = None
        if cur is not None and len(self.views) > 1 and W > 1:
            if self._comm is None:
                self._comm = torch.cuda.Stream(x.device)
            comm = self._comm

        def gather_all(j):  # chunk j of every rank, in place
            a, b, k = j * W * cr, (j + 1) * W * cr, (j * W + self.rank) * cr
            _all_gather_into(xn[a:b], xn[k:k + cr], self.group)
            _all_gather_into(rn[a:b], rn[k:k + cr], self.group)

        sent = {}  # chunk j -> its send block, written by chunk j's tail

        def send(j):
            if not (halo_out and SEND_FROM_TAIL):
                return None
            lo, hi = lay.ranges(self.rank)[j]
            sb = plan.send_block(j, lo, hi - lo, d)
            if sb is None:
                return None
            sent[j] = sb[1]
            return sb[0]

        def gather_needed(j):  # the rows the consumer reads
            if halo_out:  # straight into the consumer's halo rows
                blk = sent.pop(j, None)
                if blk is not None and x.is_cuda:  # written on the tail's stream, read on this one
                    for t in blk:
                        t.record_stream(torch.cuda.current_stream(x.device))
                exchange_halo(plan, j, xn, rn, lay.Vp, self.group,
                              gather=(lambda *_: blk) if blk is not None else None)
            else:
                exchange_rows(plan.chunks[j], xn, rn, self.group)

        def exchange(j):  # once this rank's chunk-j rows are written
            if plan is False:
                return
            self.exchanged_bytes += ((W - 1) * cr if plan is None else sum(plan.chunks[j][3])) * record_bytes(plan, d)
            if not self.collective:
                return
            fn = gather_all if plan is None else gather_needed
            if comm is None:
                fn(j)
                return
            comm.wait_stream(torch.cuda.current_stream(x.device))  # the stream chunk j's tail ran on
            with torch.cuda.stream(comm):
                fn(j)

        self._rank_launches(mode, xin, rin, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                            drop_mask, c, euclid, step, (h[:V], xn[:V], rn[:V]), gate, exchange, views=views,
                            send=send if self.collective else None)
        if comm is not None:
            cur.wait_stream(comm)
            for t in (xn, rn):
                t.record_stream(comm)
        hv, xv = h[:V], xn[:V]
        if self.collective:  # only this rank's rows of h are computed (complete_rows / fetch_rows)
            hv._regcn_owner = (self, h)
        if halo_out:  # the consumer reads the received rows at rows Vp.. (HaloView)
            xv._regcn_halo = (self.exchange_target(step), xn, rn)
        return hv, xv, rn[:V]

    # ---- owner partition: the rows other ranks computed, when a consumer needs them
    def relation_means(self, x, R2, sums_only=False):
        """Relation-context means (hyperbolic_model.relation_context) with the pairs
        partitioned like the rows: this rank sums the x rows of its own entities in every
        forward relation's r_to_e span (one sub-span per pipeline chunk), ONE all_reduce of the
        R x d sums, then / count; inverse relations copy their forward row.  sums_only: the
        rank's sums (no all_reduce, no division)."""
        R = R2 // 2
        V, d = x.shape
        wk = self.g.work()
        if self._rel is None:
            # (chunks, fixups, slots, ranges, unit weights, clamped counts): per snapshot
            ch, fx, ns, nq = self._relation_lists(R)
            self._rel = (ch, fx, ns, nq, torch.ones(R * nq, device=x.device, dtype=torch.float32),
                         wk["rel_count"][:R].clamp(min=1.0).unsqueeze(1).contiguous())
        ch, fx, ns, nq, ones, cnt = self._rel
        out = torch.zeros(R * nq, d, device=x.device, dtype=torch.float32)
        part = torch.empty(max(ns, 1), d, device=x.device, dtype=torch.float32)
        _lib.call("regcn_segment_mean_f32", _lib.fptr(x, "x"), _lib.iptr(wk["rel_idx"]), _lib.fptr(ones),
                  _lib.iptr(ch), ch.shape[0], _lib.iptr(fx), fx.shape[0], d, _lib.fptr(part), d, _lib.fptr(out),
                  _lib.stream())
        sums = out.view(R, nq, d).sum(1) if nq > 1 else out
        if sums_only:
            return sums
        if self.collective:
            allreduce_partials(sums, self.group)
        return self._relation_finish(sums, R2)

    def _relation_sums(self, x, R):
        """This rank's part of relation_means before the all_reduce: the R x d sums."""
        return ShardedGraph.relation_means(self, x, 2 * R, sums_only=True)  # not a subclass's

    def _relation_finish(self, sums, R2):
        """Means from the (all-reduced) sums; inverse relations copy their forward row."""
        R = R2 // 2
        cnt = self._rel[5]
        mean = torch.empty(R2, sums.shape[1], device=sums.device, dtype=torch.float32)  # both halves written
        torch.div(sums, cnt, out=mean[:R])
        mean[R:].copy_(mean[:R])
        return mean

    def _relation_lists(self, R):
        """(chunks, fixups, n_slots, n_ranges): every forward relation's r_to_e span cut to this
        rank's id ranges (span rows r * n_ranges + q), then at entity blocks and every 256
        pairs (graph.blocked_span_chunks)."""
        from .graph import REL_BLOCK, REL_BLOCK_CHUNK, blocked_span_chunks
        wk = self.g.work()
        dev = wk["rel_idx"].device
        ranges = self.layout.ranges(self.rank)
        rows, beg, ln = owned_rel_spans(wk["rel_idx"], wk["rel_count"][:R], ranges, self.layout.Vp)
        ch, fx, ns = blocked_span_chunks(rows, beg, ln, wk["rel_idx"], max(REL_BLOCK, 1), REL_BLOCK_CHUNK)
        _lib.publish()
        return ch, torch.from_numpy(fx).to(dev), ns, len(ranges)

    def fetch_rows(self, h, ids):
        """Make h[ids] valid on every rank (owner partition: each id's row lives on its
        owner): the owners' rows in one all_reduce of len(ids) x d (exact: every entry is
        one rank's value plus zeros), written into h."""
        meta = getattr(h, "_regcn_owner", None)
        if meta is None:
            return h
        ids = ids.to(h.device).long()
        mine = self.layout.owner(ids) == self.rank
        buf = torch.zeros(ids.numel(), h.shape[1], device=h.device, dtype=h.dtype)
        buf[mine] = h[ids[mine]]
        allreduce_partials(buf, self.group)
        h[ids] = buf
        return h

    def complete_rows(self, h):
        """All rows of a rank-local h on every rank (the full-score predict): the pipeline
        chunks' in-place all-gathers of h."""
        meta = getattr(h, "_regcn_owner", None)
        if meta is None:
            return h
        full = meta[1]
        W, cr = self.world, self.layout.cr
        for j in range(self.layout.chunks):
            a, b, k = j * W * cr, (j + 1) * W * cr, (j * W + self.rank) * cr
            _all_gather_into(full[a:b], full[k:k + cr], self.group)
        del h._regcn_owner
        return h


def complete(h):
    """h with every row valid on every rank: a rank-local state of the owner partition (the
    Poincare rows only its own launches wrote) is all-gathered in place; anything else is
    returned as is."""
    meta = getattr(h, "_regcn_owner", None)
    return meta[0].complete_rows(h) if meta is not None else h


def exposed_after(chunk_end_ms, xchg_ms):
    """The exchange time a layer exposes: exchange j starts at max(chunk j's end, exchange j-1's
    end) and takes xchg_ms[j]; the next layer starts after the last one, so the layer exposes
    end(last exchange) - end(last chunk)."""
    end = 0.0
    for tj, aj in zip(chunk_end_ms, xchg_ms):
        end = max(end, tj) + aj
    return max(0.0, end - chunk_end_ms[-1]) if chunk_end_ms else 0.0


SIM_MARKERS = os.environ.get("REGCN_SIM_MARKERS", "0") != "0"


class RankSimulation(ShardedGraph):
    """All `world` ranks of the owner partition run one after another on ONE device, for
    measurement (bench.py owner_simulation): every layer runs rank 0's chunk launches, then
    rank 1's, ... into the same output arrays (so the next layer reads valid rows, as after
    the all-gathers), each rank's launches bracketed by HIP events; the relation means sum the
    ranks' partials.  `times[k]` collects rank k's (start, end) event pairs; what a step spends
    outside them is the work every rank repeats (replicated)."""

    def __init__(self, g, world, chunks=None):
        super().__init__(g, "owner", None, 0, world, chunks)
        self.ranks = [self] + [ShardedGraph(g, "owner", None, k, world, chunks) for k in range(1, world)]
        for r in self.ranks:
            r.collective = False
        self.times = [[] for _ in range(world)]
        self.chunk_marks = [[] for _ in range(world)]  # per rank: (chunk-end events, link bytes) per layer
        self.delivery = []  # event pairs around the simulated halo deliveries (the all_to_alls' data)
        # tests: ((x block, |h|), xn, rn, send ids) of every tail-written send block
        self.keep_sends, self.sends = False, []

    def _timed(self, k, fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if SIM_MARKERS:  # profiling: a 1-cycle spin kernel around each rank's launches, so a
            torch.cuda._sleep(1)  # kernel trace tells rank work from the rest (tools/sim_replicated.py)
        a.record()
        out = fn()
        b.record()
        if SIM_MARKERS:
            torch.cuda._sleep(1)
        self.times[k].append((a, b))
        return out

    def halo_bases(self):
        """[Vp, Vp + H_0, Vp + H_0 + H_1, ...]: with every simulated rank's layers writing one
        shared buffer, rank k's halo (this snapshot as the consumer) sits at rows
        [bases[k], bases[k + 1])."""
        hit = self.__dict__.get("_halo_bases")
        if hit is None:
            sizes = [self.plan_for(k).halo.numel() for k in range(self.world)]
            hit = self.__dict__["_halo_bases"] = [self.layout.Vp + int(v) for v in np.cumsum([0] + sizes)]
        return hit

    def run_layer(self, mode, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                  drop_mask, c, euclid=False, step=None, gate=None):
        V, d = x.shape
        lay = self.layout
        tag = getattr(x, "_regcn_halo", None)
        halo_in = tag is not None and tag[0] is self
        xin, rin = (tag[1], tag[2]) if halo_in else (x, r)
        in_bases = self.halo_bases() if halo_in else None
        for sg in self.ranks:
            sg.consumers = self.consumers
        plans = [sg.exchange_plan(step) for sg in self.ranks]
        target = self.ranks[0].exchange_target(step)
        halo_out = HALO and all(isinstance(p, ExchangePlan) for p in plans)
        out_bases = target.halo_bases() if halo_out else None
        h = torch.empty(lay.Vp, d, device=x.device, dtype=torch.float32)
        xn = torch.empty(out_bases[-1] if halo_out else lay.Vp, d, device=x.device, dtype=torch.float32)
        rn = torch.empty(xn.shape[0], device=x.device, dtype=torch.float32)

        def rank_launches(k, sg, plan, marks):
            sent = {}

            def send(j):  # chunk j's send block, written by its tail
                if not (plan and halo_out and SEND_FROM_TAIL):
                    return None
                lo, hi = lay.ranges(k)[j]
                sb = plan.send_block(j, lo, hi - lo, d)
                if sb is None:
                    return None
                sent[j] = sb[1]
                if self.keep_sends:
                    self.sends.append((sb[1], xn, rn, plan.chunks[j][0]))
                return sb[0]

            def after(j):  # chunk j's rows final: the rank's send-side kernel(s) of its exchange
                if plan and halo_out:  # its send block (delivered into the halos below)
                    if sent.pop(j, None) is None:
                        gather_rows(xn, rn, plan.chunks[j][0])
                elif plan:  # the records, and the received records scattered (into scratch rows
                    sidx, _, ridx, _ = plan.chunks[j]  # here: the simulated rows hold their
                    send = pack_rows(xn, rn, sidx)      # values already)
                    recv = torch.empty(ridx.numel(), d + 4, device=x.device, dtype=torch.float32)
                    del send
                    unpack_rows(recv, ridx, scratch[0], scratch[1])
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                marks.append(e)
            views = sg.halo_views(self.plan_for(k), in_bases[k]) if halo_in else None
            sg._rank_launches(mode, xin, rin, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                              drop_mask, c, euclid, step, (h[:V], xn[:V], rn[:V]), gate, after, views=views,
                              send=send)
        scratch = None
        if not halo_out:
            scratch = self.__dict__.get("_scratch")
            if scratch is None or scratch[0].shape != xn.shape:
                scratch = self.__dict__["_scratch"] = (torch.empty_like(xn), torch.empty_like(rn))
        for k, sg in enumerate(self.ranks):
            plan = plans[k]
            marks = []
            self._timed(k, lambda: rank_launches(k, sg, plan, marks))
            rows = 0 if plan is False else ((self.world - 1) * lay.cr * lay.chunks if plan is None
                                            else plan.rows_received())
            sg.exchanged_bytes += rows * record_bytes(plan, d)
            self.chunk_marks[k].append((marks, [sg.link_bytes(plan, j, d) for j in range(len(marks))]))
        xv = xn[:V]
        if halo_out:
            # what the ranks' all_to_alls deliver on a node (RCCL over xGMI, which the link model
            # times): rank k's halo rows from their owners' rows, for the consumer's halo views;
            # bracketed so the measurement can leave it out (`delivery`)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k, p in enumerate(plans):
                a, n = out_bases[k], p.halo.numel()
                if n:
                    xn[a:a + n] = xn.index_select(0, p.halo)
                    rn[a:a + n] = rn.index_select(0, p.halo)
            e1.record()
            self.delivery.append((e0, e1))
            xv._regcn_halo = (target, xn, rn)
        return h[:V], xv, rn[:V]

    def initial_state(self, dyn, r_static, c, layer_norm):
        """Every simulated rank's initial rows (ShardedGraph.initial_state), each rank's
        launches timed as its own: own rows at their ids, its halo at rows halo_bases()[k].."""
        lay = self.layout
        V, d = dyn.shape
        bases = self.halo_bases()
        h = torch.empty(lay.Vp, d, device=dyn.device, dtype=torch.float32)
        x = torch.empty(bases[-1], d, device=dyn.device, dtype=torch.float32)
        r = torch.empty(bases[-1], device=dyn.device, dtype=torch.float32)
        for k in range(self.world):
            own, halo = self.init_rows(k)

            def launches(k=k, own=own, halo=halo):
                self._init_launch(dyn, r_static, own, own, h, x, r, c, layer_norm)
                self._init_launch(dyn, r_static, halo, None, None, x[bases[k]:], r[bases[k]:], c, layer_norm)
            self._timed(k, launches)
        xv = x[:V]
        xv._regcn_halo = (self, x, r)
        return h[:V], xv, r[:V]

    def exposed_exchange_ms(self, link_gbs=153.0):
        """Per rank: the exchange time no compute hides, summed over the layers run since
        `chunk_marks` was cleared.  Chunk j's exchange (its busiest peer link's bytes at
        `link_gbs`) starts when chunk j's rows are final and the previous exchange is done; the
        next layer starts when the last one is done, so a layer exposes end(last exchange) -
        end(last chunk)."""
        out = []
        for marks_k in self.chunk_marks:
            tot = 0.0
            for marks, nbytes in marks_k:
                if marks:
                    tot += exposed_after([marks[0].elapsed_time(e) for e in marks],
                                         [b / (link_gbs * 1e6) for b in nbytes])
            out.append(tot)
        return out


    def relation_means(self, x, R2):
        sums = [self._timed(k, lambda: ShardedGraph._relation_sums(sg, x, R2 // 2)) for k, sg in enumerate(self.ranks)]
        tot = torch.stack(sums).sum(0)  # the all_reduce of the ranks' R x d sums (one small collective)
        return ShardedGraph._relation_finish(self.ranks[0], tot, R2)

    def per_rank_ms(self):
        return [sum(a.elapsed_time(b) for a, b in t) for t in self.times]

    def delivery_ms(self):
        return sum(a.elapsed_time(b) for a, b in self.delivery)


# ------------------------------------------------------------------- sharded decoder
def combine_lse(lse_local, group=None):
    """log-sum-exp over the ranks' candidate slices of each query's per-slice lse (B floats:
    one all_gather, SURVEY.md §8(e) decoder)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return lse_local
    parts = [torch.empty_like(lse_local) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, lse_local.contiguous(), group=group)
    return torch.logsumexp(torch.stack(parts), dim=0)


def combine_counts(counts, group=None):
    """Sum of the ranks' count-greater per query (B ints: one all_reduce)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def shard_filters(filt_ptr, filt_idx, n0, n1):
    """The slice-local part [n0, n1) of a CSR list of candidate ids (shifted by -n0)."""
    ptr = np.asarray(filt_ptr, dtype=np.int64)
    idx = np.asarray(filt_idx, dtype=np.int64)
    keep = (idx >= n0) & (idx < n1)
    row = np.repeat(np.arange(len(ptr) - 1), np.diff(ptr))
    cnt = np.bincount(row[keep], minlength=len(ptr) - 1)
    new_ptr = np.zeros(len(ptr), dtype=np.int32)
    np.cumsum(cnt, out=new_ptr[1:])
    return new_ptr, (idx[keep] - n0).astype(np.int32)


class CandidateShard:
    """Rank `rank`'s contiguous slice [n0, n1) of the N all-entity candidates (SURVEY.md §8(e):
    the decoder shards its candidates; the cross entropy and the ranks need only B-sized
    exchanges), or the id `ranges` it owns (owner partition: the rows it computed).  It
    scores its candidates with the HIP scorer and combines:
      * cross entropy: per-slice log-sum-exp (regcn_hyp_ce_lse_f32 on the slice) -> combine_lse;
        the target logit is the pair score of (q_b, e_{t_b}) computed on every rank;
      * ranks: the target's score as threshold, the count of candidates above it fused into
        the scorer (regcn_hyp_rank_fused_f32: no score matrix), minus the listed answers above
        it for the filtered rank -> combine_counts, + 1.
    With group=None the collectives are skipped (a single-process simulation of one rank)."""

    def __init__(self, N, rank, world, group=None, ranges=None):
        b = even_bounds(N, world)
        self.N, self.rank, self.world, self.group = N, rank, world, group
        self.n0, self.n1 = b[rank], b[rank + 1]
        self.ranges = ranges if ranges is not None else [(self.n0, self.n1)]

    def _slice(self, cand, bias):
        c = cand[self.n0:self.n1].contiguous()
        return c, (bias[self.n0:self.n1].contiguous() if bias is not None else None)

    def scores(self, q, cand, bias, c, scale=None, margin=0.0, raw_scale=False):
        """Scores of every query against this slice, (B, n1 - n0).  raw_scale: `scale` is
        score_scale_raw (softplus on the device, as the unsharded predict scores)."""
        from .hyperbolic_decoder import _chunked_hyperbolic_dist_score
        cs, bs = self._slice(cand, bias)
        return _chunked_hyperbolic_dist_score(q, cs, bs, c, 0, 0, score_scale=scale, score_margin=margin,
                                              _raw_scale=raw_scale)

    def target_scores(self, q, cand, bias, target, c, scale=None, margin=0.0, raw_scale=False):
        """S(q_b, e_{t_b}) for every query (the diagonal of a B x B scoring of the target rows:
        the same MFMA k-order and norm order as in the full scoring, so the same bits)."""
        from .hyperbolic_decoder import _chunked_hyperbolic_dist_score
        t = target.to(cand.device).long()
        tb = bias[t].contiguous() if bias is not None else None
        S = _chunked_hyperbolic_dist_score(q, cand[t].contiguous(), tb, c, 0, 0, score_scale=scale,
                                           score_margin=margin, _raw_scale=raw_scale)  # column j carries bias[t_j]
        return torch.diagonal(S).contiguous()

    def local_lse(self, q, cand, bias, c, scale=None, margin=0.0):
        from . import _lib
        from .hyperbolic_decoder import _scalar
        cs, bs = self._slice(cand, bias)
        B, d = q.shape
        n = cs.shape[0]
        q = q.contiguous().float()
        tgt = torch.full((B,), -1, device=q.device, dtype=torch.int32)  # no target logit needed here
        ws = torch.empty((_lib.lib().regcn_hyp_ce_workspace_bytes(B, n) + 3) // 4, device=q.device)
        loss = torch.empty(B, device=q.device)
        lse = torch.empty(B, device=q.device)
        f = _lib.fptr
        sc = _scalar(scale if scale is not None else 1.0, q)
        mg = _scalar(margin, q)
        _lib.call("regcn_hyp_ce_lse_f32", f(q, "query"), f(cs, "candidates"), f(bs), f(sc), f(mg), _lib.iptr(tgt),
                  B, n, d, float(c), 0, f(ws), f(loss), f(lse), _lib.stream())
        return lse

    def ce_loss(self, q, cand, target, c, bias=None, scale=None, margin=0.0):
        """mean_b (lse_b - S(q_b, e_{t_b})) over all N candidates (replicated on every rank)."""
        lse = combine_lse(self.local_lse(q, cand, bias, c, scale, margin), self.group)
        return (lse - self.target_scores(q, cand, bias, target, c, scale, margin)).mean()

    def local_counts(self, local_scores, ts, filt_ptr=None, filt_idx=None):
        from . import _lib
        B, n = local_scores.shape
        dev = local_scores.device
        raw = torch.empty(B, device=dev, dtype=torch.int32)
        flt = torch.empty(B, device=dev, dtype=torch.int32)
        fp = fi = None
        if filt_ptr is not None:
            p_, i_ = shard_filters(filt_ptr, filt_idx, self.n0, self.n1)
            fp = torch.from_numpy(p_).to(dev)
            fi = torch.from_numpy(i_).to(dev) if len(i_) else torch.zeros(1, device=dev, dtype=torch.int32)
        _lib.call("regcn_rank_count_f32", _lib.fptr(local_scores.contiguous(), "score"), B, n,
                  _lib.fptr(ts.contiguous().float(), "threshold"), _lib.iptr(fp), _lib.iptr(fi), _lib.iptr(raw),
                  _lib.iptr(flt) if fp is not None else None, _lib.stream())
        return raw, (flt if fp is not None else None)

    def ranks(self, local_scores, ts, filt_ptr=None, filt_idx=None):
        """(rank, filtered rank) over all N candidates, 1-based, replicated."""
        raw, flt = self.local_counts(local_scores, ts, filt_ptr, filt_idx)
        both = torch.stack([raw, flt if flt is not None else raw])
        both = combine_counts(both, self.group)
        return both[0].long() + 1, both[1].long() + 1

    def fused_counts(self, q, cand, bias, c, ts, scale=None, margin=0.0, raw_scale=False):
        """#{n in this shard's id ranges : S(q_b, e_n) > ts_b} with no score matrix and no copy
        of the candidate rows: regcn_hyp_rank_fused_f32 over the ranges (up to 8 per launch, the
        counts accumulated on the device).  S is bit for bit the full scoring's, so the counts
        equal regcn_rank_count_f32's over the score matrix.  None when the fused scorer does
        not apply (d % 4 != 0 or d > 256)."""
        from .hyperbolic_decoder import _scalar
        B, d = q.shape
        if d % 4 or d > 256:
            return None
        dev = q.device
        q = q.contiguous().float()
        cand = cand.contiguous()
        ts = ts.contiguous().float()
        counts = torch.zeros(B, device=dev, dtype=torch.int32)
        spans = [(a, b) for a, b in self.ranges if b > a]
        if not spans or B == 0:
            return counts
        N = cand.shape[0]
        ws = torch.empty((_lib.lib().regcn_hyp_ce_workspace_bytes(B, N) + 3) // 4, device=dev)
        sc = _scalar(scale if scale is not None else 1.0, q)
        mg = _scalar(margin, q)
        flags = _lib.SCORE_RAW_SCALE if raw_scale else 0
        f = _lib.fptr
        for k in range(0, len(spans), 8):
            part = spans[k:k + 8]
            rng = (ctypes.c_int32 * (2 * len(part)))(*[v for ab in part for v in ab])
            _lib.call("regcn_hyp_rank_fused_f32", f(q, "query"), f(cand, "candidates"), f(bias), f(sc), f(mg),
                      f(ts, "threshold"), B, N, d, float(c), flags, rng, len(part), f(ws), int(k > 0),
                      _lib.iptr(counts), _lib.stream())
        return counts

    def filter_hits(self, q, cand, bias, c, ts, filt_ptr, filt_idx, **kw):
        """#{f in query b's filter list, f in this shard's ranges : S(q_b, e_f) > ts_b}: the
        filtered count is the raw count minus these.  The listed candidates are scored as one
        block (the same per-pair bits as the full scoring) and compared on the device."""
        from .hyperbolic_decoder import _chunked_hyperbolic_dist_score
        ptr = np.asarray(filt_ptr, dtype=np.int64)
        idx = np.asarray(filt_idx, dtype=np.int64)
        row = np.repeat(np.arange(len(ptr) - 1), np.diff(ptr))
        keep = np.zeros(len(idx), dtype=bool)
        for a, b in self.ranges:
            keep |= (idx >= a) & (idx < b)
        B = q.shape[0]
        dev = q.device
        if not keep.any():
            return torch.zeros(B, device=dev, dtype=torch.int32)
        row, idx = row[keep], idx[keep]
        uniq, pos = np.unique(idx, return_inverse=True)
        u = torch.from_numpy(uniq).to(dev)
        S = _chunked_hyperbolic_dist_score(q, cand.index_select(0, u), bias.index_select(0, u) if bias is not None
                                           else None, c, 0, 0, score_scale=kw.get("scale"),
                                           score_margin=kw.get("margin", 0.0), _raw_scale=kw.get("raw_scale", False))
        rt = torch.from_numpy(row).to(dev)
        hit = (S[rt, torch.from_numpy(pos).to(dev)] > ts.float()[rt]).to(torch.int32)
        return torch.zeros(B, device=dev, dtype=torch.int32).index_add_(0, rt, hit)

    def range_ranks(self, q, cand, bias, c, ts, filt_ptr=None, filt_idx=None, **kw):
        """(rank, filtered rank) over all N candidates, 1-based, replicated: this shard's counts
        over its id ranges (fused_counts: no score matrix; the filtered count subtracts
        filter_hits), then ONE all_reduce of the 2B counts.  Without the fused scorer: one
        scorer launch and one count launch per range."""
        raw = self.fused_counts(q, cand, bias, c, ts, **kw)
        if raw is not None:
            flt = raw - self.filter_hits(q, cand, bias, c, ts, filt_ptr, filt_idx, **kw) if filt_ptr is not None \
                else raw
            tot = combine_counts(torch.stack([raw, flt]), self.group)
            return tot[0].long() + 1, tot[1].long() + 1
        tot = None
        for n0, n1 in self.ranges:
            self.n0, self.n1 = n0, n1
            raw, flt = self.local_counts(self.scores(q, cand, bias, c, **kw), ts, filt_ptr, filt_idx)
            both = torch.stack([raw, flt if flt is not None else raw])
            tot = both if tot is None else tot + both
        if tot is None:
            tot = torch.zeros(2, q.shape[0], device=q.device, dtype=torch.int32)
        tot = combine_counts(tot, self.group)
        return tot[0].long() + 1, tot[1].long() + 1


# ------------------------------------------------------------------ training replicas
def allreduce_gradients(params, group=None):
    """Data-parallel training (replicas process different (history window,
    target snapshot) samples): average every parameter gradient over the ranks with ONE
    all-reduce of the flattened gradients (~2.5-2.8M floats for the reference models: a
    single bucket, sized for point-to-point xGMI rather than per-tensor calls).

    A per-parameter has-gradient flag travels in the same bucket.  A parameter no rank
    produced a gradient for keeps `grad = None`, exactly as in a single process, so the
    optimizer skips it (Adam's weight decay would otherwise move it by ~lr per step); one
    that only some ranks touched gets the mean over all ranks, the others contributing
    zeros.  Returns the number of floats reduced."""
    params = [p for p in params if p.requires_grad]
    if not (dist.is_initialized() and dist.get_world_size(group) > 1) or not params:
        return 0
    world = dist.get_world_size(group)
    dev = params[0].device
    has = torch.tensor([1.0 if p.grad is not None else 0.0 for p in params], device=dev)
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params]
                     + [has])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flags = flat[-len(params):].tolist()
    flat = flat[:-len(params)].div_(world)
    off = 0
    for p, f in zip(params, flags):
        n = p.numel()
        if f > 0:
            g = flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
        else:
            p.grad = None
        off += n
    return int(flat.numel())


def broadcast_state(module, src=0, group=None):
    """Replicas start from rank `src`'s parameters and buffers (one broadcast per tensor at
    start-up; the per-step traffic is allreduce_gradients)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    # into the tensors themselves (not through `.data`): the in-place write bumps each
    # tensor's version counter, which the parameter-derived caches are keyed on
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src, group=group)
    from .weights import invalidate
    invalidate(module)
