"""Multi-GPU partitions of one snapshot, one process per GPU, RCCL.

Two partitionings of a message-passing layer over `world` ranks:

* ``"edge"`` — the north star's literal scheme: rank k aggregates the k-th contiguous slice
  of the destination-sorted edge list (balanced by edge count) into raw per-row partial
  sums (union: sum_e w_e (x_src + rel); Lorentz: the summed Lorentz points plus their
  time coordinate); one ``all_reduce(SUM)`` of the V x (d + 1) partials; every rank
  finishes the rows (norm / centroid -> log0) and runs the MFMA tail on all rows.
* ``"owner"`` — rank k owns the k-th contiguous block of ceil(V / world) destination nodes
  and runs the fused layer kernel on them only (gather + GEMMs + epilogue, rank-local);
  an ``all_gather`` of the owned rows of (h, log0 h, |h|) rebuilds the full state.

`ShardedGraph` wraps a `SnapshotGraph` with one of the two; the HIP layers dispatch on it,
so `HyperbolicRecurrentRGCN.forward(g_list=[ShardedGraph, ...])` runs sharded.  The
collective helpers (`allreduce_partials`, `allgather_rows`) and the plans are plain
torch.distributed / numpy, covered on CPU with gloo (tests/test_parallel.py); the compute
between them is the HIP library (tests/test_gpu_parity.py simulates the ranks on one GPU).
"""
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
        h = g._host
        rowptr = h["rowptr"].astype(np.int64)
        V = g.number_of_nodes()
        E = int(rowptr[-1])
        self.e0, self.e1 = even_bounds(E, world)[rank:rank + 2]
        ce = g.chunk_edges
        rows = np.nonzero((rowptr[:-1] < self.e1) & (rowptr[1:] > self.e0))[0]
        beg = np.maximum(rowptr[rows], self.e0)
        end = np.minimum(rowptr[rows + 1], self.e1)
        chunks, fix, slot = [], [], 0
        for r, b, e in zip(rows.tolist(), beg.tolist(), end.tolist()):
            k = (e - b + ce - 1) // ce
            for i in range(k):
                chunks.append((r, b + i * ce, min(b + (i + 1) * ce, e), slot + i))
            fix.append((r, slot, slot + k, 0))
            slot += k
        self.chunks = np.asarray(chunks, dtype=np.int32).reshape(-1, 4)
        self.fixups, self.n_slots = group_fixups(fix, slot)
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


class OwnerView:
    """A rank's view of a snapshot under the owner partition: the global CSR and relation
    spans, and the fused-kernel work lists of its node block only."""

    def __init__(self, g, rank, world):
        self.g = g
        self.per, b = owner_bounds(g.number_of_nodes(), world)
        self.v0, self.v1 = b[rank], b[rank + 1]
        h = g._host
        fw = fused_work(np.arange(self.v0, self.v1), g.in_deg_np, h["rowptr"].astype(np.int64),
                        h["col_src"].astype(np.int64), h["col_type"].astype(np.int64), g.budget, g.pack_items,
                        g.chunk_edges)
        self.fw = fw
        self.budget, self.n_pos, self.n_pos_tiles = g.budget, fw.n_pos, fw.n_pos_tiles
        self.n_heavy, self.heavy_slots = fw.n_heavy, fw.heavy_slots
        self._dev = None

    def work(self):
        if self._dev is None:
            wk = dict(self.g.work())
            dev = wk["rowptr"].device
            wk.update({k: torch.from_numpy(v).to(dev) for k, v in self.fw.host.items()})
            self._dev = wk
        return self._dev


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
        dist.all_gather_into_tensor(full, chunk, group=group)
    return full


# ---------------------------------------------------------------------- sharded layers
class ShardedGraph:
    """A SnapshotGraph partitioned across the ranks of `group` (see module docstring).
    Everything but the message-passing layers (relation spans, degrees, ...) is the
    wrapped graph's."""

    def __init__(self, g, partition="owner", group=None, rank=None, world=None):
        if partition not in ("edge", "owner"):
            raise ValueError("partition must be 'edge' or 'owner'")
        self.g, self.partition, self.group = g, partition, group
        if rank is None:
            rank = dist.get_rank(group) if dist.is_initialized() else 0
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank, self.world = rank, world
        self.plan = EdgePlan(g, rank, world).to(g.device) if partition == "edge" else None
        self.view = OwnerView(g, rank, world) if partition == "owner" else None

    def __getattr__(self, name):  # delegate the DGL-visible surface and work lists
        return getattr(self.__dict__["g"], name)

    def work(self):
        return self.g.work()

    def to(self, device):
        device = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        if device == self.g.device:
            return self
        return ShardedGraph(self.g.to(device), self.partition, self.group, self.rank, self.world)

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
            _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(w_rel), i(wk["col_src"]), i(wk["col_type"]),
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

    def run_layer(self, mode, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                  drop_mask, c, euclid=False, step=None):
        """The sharded counterpart of hyperbolic_layers.run_layer (same arguments/returns)."""
        from .hyperbolic_layers import run_layer
        V, d = x.shape
        if self.partition == "edge":
            P = self.edge_partials(mode, x, r, rel, w_rel, nb, gamma, c)
            allreduce_partials(P, self.group)
            agg = self.edge_finish(mode, P, x, r, rel, w_rel, nb, gamma, c)
            return run_layer(_lib.AGG_NONE, self.g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t,
                             w_skip, b_skip, drop_mask, c, euclid=euclid, step=step, agg=agg)
        per = self.view.per
        Vp = per * self.world
        h = torch.empty(Vp, d, device=x.device, dtype=torch.float32)
        xn = torch.empty(Vp, d, device=x.device, dtype=torch.float32)
        rn = torch.empty(Vp, device=x.device, dtype=torch.float32)
        run_layer(mode, self.view, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                  drop_mask, c, euclid=euclid, step=step, out=(h[:V], xn[:V], rn[:V]))
        for t in (h, xn, rn):
            allgather_rows(t, per, self.group)
        return h[:V], xn[:V], rn[:V]
