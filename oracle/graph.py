"""Snapshot-graph construction restated (oracle; test infrastructure only).

Follows rgcn/utils.py:78-134 (`r2e`, `build_sub_graph`).
"""
import numpy as np


def r2e(triples, num_rels):
    """rgcn/utils.py:78-97.

    uniq_r = unique(r) ++ unique(r)+R; r_to_e[r] = set of s and o of triples
    with relation r (the inverse id shares the forward set).  The reference
    emits each set in Python set-iteration order; here each span is sorted,
    so spans must be compared as sets.
    Returns (uniq_r int64 (U,), r_len int64 (U,2), r_to_e int64 (sum,)).
    """
    triples = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    src, rel, dst = triples[:, 0], triples[:, 1], triples[:, 2]
    uniq = np.unique(rel)
    uniq_r = np.concatenate([uniq, uniq + num_rels])
    ents = {}
    for r in uniq:
        m = rel == r
        ents[int(r)] = np.unique(np.concatenate([src[m], dst[m]]))
    spans, flat, idx = [], [], 0
    for r in uniq_r:
        e = ents[int(r) % num_rels if r >= num_rels else int(r)]
        spans.append((idx, idx + len(e)))
        flat.append(e)
        idx += len(e)
    r_to_e = np.concatenate(flat) if flat else np.zeros(0, np.int64)
    return uniq_r.astype(np.int64), np.asarray(spans, dtype=np.int64).reshape(-1, 2), r_to_e


def row_subgraph(num_nodes, num_rels, triples, rows):
    """build_sub_graph restricted to the in-edges of `rows` (for pinning single rows of a graph
    too large for the whole-graph oracle): the edges whose destination is in `rows`, in the
    reference's order, relabelled onto the compact node list `nodes` = rows followed by the
    other sources; in_deg / norm are the full graph's (rgcn/utils.py:110-114), so the rows'
    layer outputs equal the whole-graph ones.  Returns (g, nodes)."""
    triples = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    rows = np.asarray(rows, dtype=np.int64)
    s, r, o = triples[:, 0], triples[:, 1], triples[:, 2]
    in_deg = np.bincount(o, minlength=num_nodes) + np.bincount(s, minlength=num_nodes)
    pick = np.zeros(num_nodes, bool)
    pick[rows] = True
    fwd, inv = pick[o], pick[s]
    src = np.concatenate([s[fwd], o[inv]])
    dst = np.concatenate([o[fwd], s[inv]])
    etype = np.concatenate([r[fwd], r[inv] + num_rels])
    extra = np.setdiff1d(np.unique(src), rows)
    nodes = np.concatenate([rows, extra])
    pos = np.full(num_nodes, -1, np.int64)
    pos[nodes] = np.arange(nodes.size)
    deg = in_deg[nodes].astype(np.int64)
    deg_f = deg.astype(np.float32)
    deg_f[deg_f == 0] = 1.0
    norm = (np.float32(1.0) / deg_f).astype(np.float32)
    return {"num_nodes": int(nodes.size), "src": pos[src], "dst": pos[dst], "type": etype, "in_deg": deg,
            "norm": norm}, nodes


def build_sub_graph(num_nodes, num_rels, triples):
    """rgcn/utils.py:100-134 restated without DGL.

    Edges (in the reference's order): src=cat(s,o), dst=cat(o,s),
    type=cat(r, r+R) (:116-118, :125).  in_deg counts the doubled graph;
    norm = 1/in_deg with 0 -> 1, fp32 (:110-114); edge norm = norm[dst]*norm[src]
    (:124); node id = arange(V) (:122).
    """
    triples = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
    s, r, o = triples[:, 0], triples[:, 1], triples[:, 2]
    src = np.concatenate([s, o])
    dst = np.concatenate([o, s])
    etype = np.concatenate([r, r + num_rels])
    in_deg = np.bincount(dst, minlength=num_nodes).astype(np.int64)
    deg_f = in_deg.astype(np.float32)
    deg_f[deg_f == 0] = 1.0
    norm = (np.float32(1.0) / deg_f).astype(np.float32)
    enorm = (norm[dst] * norm[src]).astype(np.float32)
    uniq_r, r_len, r_to_e = r2e(triples, num_rels)
    return {
        "num_nodes": int(num_nodes), "src": src, "dst": dst, "type": etype, "in_deg": in_deg,
        "norm": norm, "enorm": enorm, "uniq_r": uniq_r, "r_len": r_len, "r_to_e": r_to_e,
    }
