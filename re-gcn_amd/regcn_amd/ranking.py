"""Evaluation ranking with time-aware filtering (mirror of rgcn/utils.py:21-305, SURVEY.md
§8(f) row f2).

`get_total_rank(test_triples, score, all_ans, eval_bz, rel_predict=0)` keeps the reference
signature and returns `(filter_mrr, mrr, rank, filter_rank)`, but instead of two full
`torch.sort`s per batch and a host loop writing -1e7 into the filtered answers it runs one
HIP kernel (`regcn_rank_f32`): rank = 1 + #{candidates scoring strictly above the target},
and the filtered rank additionally excludes the other true answers of the same snapshot
(a CSR list built once on the host).  Without score ties against the target this equals
the reference's sort position + 1; with ties the reference's order is whatever
`torch.sort` returns (unspecified), the kernel counts the tie as not above (the optimistic
rank).  As in the reference (filter_score / filter_score_r write into a view of `score`,
rgcn/utils.py:51-75), `score` leaves get_total_rank with the other true answers set to
-1e7, so `construct_snap` under --multi-step picks its top-k from the filtered scores.
"""
import numpy as np
import torch

from . import _lib


def _filter_csr(test_triples, all_ans, rel_predict):
    """Per query, the other true answers (reference filter_score / filter_score_r)."""
    tri = test_triples.detach().cpu().numpy()
    ptr = [0]
    idx = []
    for h, r, t in tri.tolist():
        if all_ans is None:
            ans = ()
        elif rel_predict:
            ans = set(all_ans.get(h, {}).get(t, ())) - {r}
        else:
            ans = set(all_ans.get(h, {}).get(r, ())) - {t}
        idx.extend(sorted(ans))
        ptr.append(len(idx))
    return np.asarray(ptr, dtype=np.int32), np.asarray(idx, dtype=np.int32)


def ranks(score, target, filt_ptr=None, filt_idx=None):
    """(rank, filtered rank), 1-based int64, one HIP launch."""
    B, N = score.shape
    s = score.detach().contiguous().float()
    dev = s.device
    tgt = target.to(device=dev, dtype=torch.int32).contiguous()
    raw = torch.empty(B, device=dev, dtype=torch.int32)
    flt = torch.empty(B, device=dev, dtype=torch.int32)
    fp = torch.from_numpy(filt_ptr).to(dev) if filt_ptr is not None else None
    fi = torch.from_numpy(filt_idx).to(dev) if filt_idx is not None and len(filt_idx) else None
    if fp is not None and fi is None:  # no other answers anywhere: empty lists
        fi = torch.zeros(1, device=dev, dtype=torch.int32)
    _lib.call("regcn_rank_f32", _lib.fptr(s, "score"), B, N, _lib.iptr(tgt, "target"), _lib.iptr(fp), _lib.iptr(fi),
              _lib.iptr(raw), _lib.iptr(flt), _lib.stream())
    return raw.long(), flt.long()


FILTERED_SCORE = -10000000.0  # rgcn/utils.py:60, :74


def apply_filter_(score, filt_ptr, filt_idx):
    """Write -1e7 into `score[b, filt_idx[filt_ptr[b]:filt_ptr[b+1]]]` in place, as
    filter_score / filter_score_r do (rgcn/utils.py:51-75): one device index_put."""
    if filt_idx is None or len(filt_idx) == 0:
        return score
    counts = np.diff(filt_ptr).astype(np.int64)
    rows = torch.from_numpy(np.repeat(np.arange(len(counts), dtype=np.int64), counts)).to(score.device)
    cols = torch.from_numpy(filt_idx.astype(np.int64)).to(score.device)
    score[rows, cols] = FILTERED_SCORE
    return score


def sort_and_rank(score, target):
    """rgcn/utils.py:21-25: 0-based position of the target among the candidates."""
    return ranks(score, target)[0] - 1


def get_total_rank(test_triples, score, all_ans, eval_bz, rel_predict=0):
    """rgcn/utils.py:136-166.  eval_bz only batched the reference's sorts; one launch here."""
    col = {1: 1, 2: 0}.get(int(rel_predict), 2)
    target = test_triples[:, col]
    fp, fi = _filter_csr(test_triples, all_ans, bool(rel_predict))
    rank, filter_rank = ranks(score, target, fp, fi)
    apply_filter_(score, fp, fi)
    mrr = torch.mean(1.0 / rank.float())
    filter_mrr = torch.mean(1.0 / filter_rank.float())
    return filter_mrr.item(), mrr.item(), rank, filter_rank


def stat_ranks(rank_list, method):
    """rgcn/utils.py:169-178."""
    total_rank = torch.cat(rank_list)
    mrr = torch.mean(1.0 / total_rank.float())
    print("MRR ({}): {:.6f}".format(method, mrr.item()))
    for hit in (1, 3, 10):
        print("Hits ({}) @ {}: {:.6f}".format(method, hit, torch.mean((total_rank <= hit).float()).item()))
    return mrr


def construct_snap(test_triples, num_nodes, num_rels, final_score, topK):
    """rgcn/utils.py:367-381: the top-k predicted objects as next-history triples."""
    _, idx = torch.sort(final_score, dim=1, descending=True)
    top = idx[:, :topK].cpu().numpy()
    tri = test_triples.cpu().numpy()
    out = []
    for (h, r, _), cand in zip(tri.tolist(), top.tolist()):
        for o in cand:
            out.append([h, r, o] if r < num_rels else [o, r - num_rels, h])
    return np.array(out, dtype=int).reshape(-1, 3)


def construct_snap_r(test_triples, num_nodes, num_rels, final_score, topK):
    """rgcn/utils.py:383-406: the top-k predicted relations as next-history triples."""
    _, idx = torch.sort(final_score, dim=1, descending=True)
    top = idx[:, :topK].cpu().numpy()
    tri = test_triples.cpu().numpy()
    out = []
    for (h, _, t), cand in zip(tri.tolist(), top.tolist()):
        for r in cand:
            out.append([h, r, t] if r < num_rels else [t, r - num_rels, h])
    return np.array(out, dtype=int).reshape(-1, 3)


def load_all_answers_for_filter(total_data, num_rel, rel_p=False):
    """rgcn/utils.py:264-283: {s: {r: {o}}, o: {r + R: {s}}} (or {s: {o: {r}}} for
    relation prediction) over one snapshot's triples."""
    all_ans = {}
    for s, r, o in np.asarray(total_data)[:, :3].tolist():
        if rel_p:
            all_ans.setdefault(s, {}).setdefault(o, set()).add(r)
            all_ans.setdefault(o, {}).setdefault(s, set()).add(r + num_rel)
        else:
            all_ans.setdefault(o, {}).setdefault(r + num_rel, set()).add(s)
            all_ans.setdefault(s, {}).setdefault(r, set()).add(o)
    return all_ans


def split_by_time(data):
    """rgcn/utils.py:306-339: consecutive runs of equal time (column 3; the data is in time
    order, as the reference requires) as (s, r, o) snapshots."""
    data = np.asarray(data)
    if len(data) == 0:
        return []
    cuts = np.nonzero(np.diff(data[:, 3]))[0] + 1
    return [chunk[:, :3].copy() for chunk in np.split(data, cuts)]


def load_all_answers_for_time_filter(total_data, num_rels, num_nodes, rel_p=False):
    """rgcn/utils.py:286-303: one filter dict per snapshot."""
    return [load_all_answers_for_filter(snap, num_rels, rel_p) for snap in split_by_time(total_data)]
