"""Synthetic temporal KG snapshots shaped like the datasets BASELINE.json names.

The datasets (ICEWS14s, ICEWS18, GDELT) are absent, so every config runs on
snapshots with the named |V|, |R| and triples/snapshot:
  * subjects/objects Zipf(alpha=1.1) over a random permutation of the entities,
    relations uniform;
  * temporal signal: a fraction 0.6 of each snapshot's triples is resampled from the
    previous 1-3 snapshots, so the recurrence is learnable.
"""
import numpy as np

CONFIGS = {
    # name: (V, R, triples per snapshot, history T, encoder, decoder, n_bases)
    "icews14s_lgcn_roth": dict(V=7128, R=230, per_snap=246, T=3, encoder="lgcn", decoder="roth", n_bases=100,
                               label="ICEWS14s hyperbolic: encoder=lgcn, decoder=roth, c=0.01, d=200"),
    "icews14s_uvrgcn_convtranse": dict(V=7128, R=230, per_snap=246, T=3, encoder="uvrgcn", decoder="convtranse",
                                       n_bases=100, label="ICEWS14s RE-GCN uvrgcn + convtranse, d=200"),
    "icews18_roth": dict(V=23033, R=256, per_snap=1540, T=3, encoder="hyperbolic_uvrgcn", decoder="roth",
                         n_bases=100, label="ICEWS18, d=200, n-layers=2, decoder=roth"),
    "gdelt": dict(V=7691, R=240, per_snap=770, T=7, encoder="hyperbolic_uvrgcn", decoder="roth", n_bases=100,
                  label="GDELT, d=200, history_len=7"),
    "synthetic_1m": dict(V=1_000_000, R=256, per_snap=25_000_000, T=3, encoder="hyperbolic_uvrgcn",
                         decoder="roth", n_bases=100, scale=True,
                         label="Synthetic TKG |V|=1M, |E|=50M/snapshot, |R|=256, d=200"),
}


def zipf_triples(rng, V, R, n, alpha=1.1, perm=None, uniform_s=False):
    """n triples: objects (and subjects unless `uniform_s`) Zipf(alpha) over `perm`, subjects
    uniform with `uniform_s` (the HBM-honest gather variant: the hub rows' in-edges then come
    from uniformly spread sources, SURVEY.md §8(d) load-balance A/B), relations uniform."""
    perm = rng.permutation(V) if perm is None else perm
    # inverse-CDF sampling of a truncated Zipf law (no V-sized probability table per call)
    u = rng.random(2 * n)
    ranks = np.floor(((V ** (1 - alpha) - 1) * u + 1) ** (1 / (1 - alpha))).astype(np.int64) - 1
    ranks = np.clip(ranks, 0, V - 1)
    s, o = perm[ranks[:n]], perm[ranks[n:]]
    if uniform_s:
        s = rng.integers(0, V, size=n)
    r = rng.integers(0, R, size=n)
    return np.stack([s, r, o], 1).astype(np.int64)


def snapshot_series(seed, V, R, n_snap, per_snap, recur=0.6, uniform_s=False):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(V)
    snaps = []
    for _ in range(n_snap):
        tr = zipf_triples(rng, V, R, per_snap, perm=perm, uniform_s=uniform_s)
        if snaps and recur > 0:
            k = int(recur * per_snap)
            pool = np.concatenate(snaps[-3:])
            tr[:k] = pool[rng.integers(0, len(pool), size=k)]
        snaps.append(tr)
    return snaps
