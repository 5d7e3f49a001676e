"""Test-only stand-in for the subset of DGL 0.5.2 the reference touches.

CONTAINER ONLY: used by tools/goldens/make_golden.py to import /root/reference
(which imports `dgl`) and generate golden vectors.  Never shipped, never used by
the product package, never present on the GPU box path.

It restates DGL's documented message-passing semantics (not DGL's code):
  * update_all(msg, builtin sum, apply): per-edge messages are summed into
    their destination; nodes without in-edges receive zeros; the apply
    function then runs on every node.
  * update_all(msg, udf_reduce, apply): destinations are bucketed by in-degree
    and the reducer sees a mailbox (n_nodes, degree, ...) whose second axis
    follows edge-id order; zero-in-degree nodes receive zeros.
"""
import torch
from . import function  # noqa: F401


class _Frame(dict):
    pass


class _EdgeBatch:
    def __init__(self, g, eids):
        self._g, self._eids = g, eids
        src, dst = g._src[eids], g._dst[eids]
        self.src = {k: v[src] for k, v in g.ndata.items()}
        self.dst = {k: v[dst] for k, v in g.ndata.items()}
        self.data = {k: v[eids] for k, v in g.edata.items()}


class _NodeBatch:
    def __init__(self, data, mailbox=None):
        self.data = data
        self.mailbox = mailbox


class DGLGraph:
    def __init__(self, src, dst, num_nodes):
        self._src = torch.as_tensor(src, dtype=torch.long)
        self._dst = torch.as_tensor(dst, dtype=torch.long)
        self._n = int(num_nodes)
        self.ndata = _Frame()
        self.edata = _Frame()

    def number_of_nodes(self):
        return self._n

    def number_of_edges(self):
        return int(self._src.numel())

    def in_degrees(self, v=None):
        deg = torch.bincount(self._dst, minlength=self._n)
        if v is None:
            return deg
        idx = torch.as_tensor(list(v) if isinstance(v, range) else v, dtype=torch.long)
        return deg[idx]

    def to(self, device):
        dev = torch.device(device) if not isinstance(device, torch.device) else device
        g = DGLGraph(self._src.to(dev), self._dst.to(dev), self._n)
        g.ndata.update({k: v.to(dev) for k, v in self.ndata.items()})
        g.edata.update({k: v.to(dev) for k, v in self.edata.items()})
        for k, v in self.__dict__.items():
            if k not in ("_src", "_dst", "_n", "ndata", "edata"):
                setattr(g, k, v)
        return g

    def apply_edges(self, func):
        out = func(_EdgeBatch(self, torch.arange(self.number_of_edges())))
        self.edata.update(out)

    def update_all(self, message_func, reduce_func, apply_node_func=None):
        n, E = self._n, self.number_of_edges()
        msgs = message_func(_EdgeBatch(self, torch.arange(E, device=self._src.device)))
        new = {}
        if isinstance(reduce_func, function._SumReducer):
            m = msgs[reduce_func.msg]
            acc = torch.zeros((n,) + tuple(m.shape[1:]), dtype=m.dtype, device=m.device)
            acc.index_add_(0, self._dst, m)
            new[reduce_func.out] = acc
        else:
            deg = torch.bincount(self._dst, minlength=n)
            order = torch.argsort(self._dst * (E + 1) + torch.arange(E, device=self._dst.device))
            dst_sorted = self._dst[order]
            starts = torch.zeros(n + 1, dtype=torch.long)
            starts[1:] = torch.cumsum(deg.cpu(), 0)
            outs = None
            for d in sorted(set(deg.tolist()) - {0}):
                nodes = torch.nonzero(deg == d, as_tuple=False).view(-1)
                eidx = torch.stack([order[starts[v]:starts[v] + d] for v in nodes.tolist()])
                mailbox = {k: v[eidx] for k, v in msgs.items()}
                data = {k: v[nodes] for k, v in self.ndata.items()}
                res = reduce_func(_NodeBatch(data, mailbox))
                if outs is None:
                    outs = {k: torch.zeros((n,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                            for k, v in res.items()}
                for k, v in res.items():
                    outs[k][nodes] = v
            new = outs or {}
            del dst_sorted
        self.ndata.update(new)
        if apply_node_func is not None:
            self.ndata.update(apply_node_func(_NodeBatch(dict(self.ndata))))


def graph(data, num_nodes=None):
    src, dst = data
    src = torch.as_tensor(src, dtype=torch.long)
    dst = torch.as_tensor(dst, dtype=torch.long)
    if num_nodes is None:
        num_nodes = int(max(src.max(), dst.max())) + 1
    return DGLGraph(src, dst, num_nodes)
