"""--run-analysis statistics (hyperbolic_main.py:716; SURVEY.md §5 "metrics / observability").

The reference collects, when `analysis=True`:
  * per timestep, the time gate tensor and its mean (gate_list / training_stats
    ["time_gate_values"], hyperbolic_model.py:852-856, :887-888);
  * the radius evolution's last statistics (TemporalRadiusEvolution.last_evolution_stats,
    hyperbolic_ops.py:426-434);
  * embedding-norm statistics of the initial and the predicted embeddings
    (HyperbolicOps.log_embedding_stats, hyperbolic_ops.py:235-269; hyperbolic_model.py:791-792,
    :932-933);
  * the loss components of every get_loss (:1076-1082) and the total gradient norm of
    log_gradient_stats (:1090-1108), summarised by get_training_summary (:1110-1127).
Each of those reads a device value with `.item()` the moment it is produced.  Here every
statistic stays a device tensor when produced (the per-element time gates and radius terms come
out of the analysis variant of the timestep kernel, regcn_timestep_analysis_f32) and is read on
the host only where a caller looks at it: TrainingStats materialises on access,
get_evolution_stats / get_training_summary once per call.  Debug log lines that print values
are only formatted (and so only synchronise) when the logger is enabled for DEBUG.
"""
import logging

import torch

logger = logging.getLogger("hyperbolic_model")


def _host(v):
    """Device tensors / nested containers of them -> python numbers (one read per tensor)."""
    if torch.is_tensor(v):
        return v.item() if v.numel() == 1 else v.tolist()
    if isinstance(v, dict):
        return {k: _host(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_host(x) for x in v)
    return v


class TrainingStats(dict):
    """model.training_stats (hyperbolic_model.py:307-312): the same keys; values are kept as
    device tensors and read as python numbers / lists when accessed."""

    def __init__(self):
        super().__init__(embedding_norms=[], gradient_norms=[], loss_components=[], time_gate_values=[])

    def raw(self, key):
        return dict.__getitem__(self, key)

    def __getitem__(self, key):
        return _host(dict.__getitem__(self, key))

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]

    def __repr__(self):
        return repr(dict(self.items()))


def evolution_terms(delta, dyn, base, r_static, beta, eps):
    """TemporalRadiusEvolution.last_evolution_stats (hyperbolic_ops.py:426-434) from the per-row
    clipped delta, dynamic radius, base radius and the static radius, as ONE device vector
    [delta_mean, delta_std, dynamic_radius_mean, static_radius_mean, base_radius_mean] (std
    unbiased, as torch.std) plus the two constants."""
    vec = torch.stack([delta.mean(), delta.std(), dyn.mean(), r_static.mean(), base.mean()]).detach()
    return {"vec": vec, "anchor_beta": float(beta), "epsilon": float(eps)}


EVOLUTION_KEYS = ("delta_mean", "delta_std", "dynamic_radius_mean", "static_radius_mean", "base_radius_mean")


def evolution_dict(ev):
    """The host dict get_evolution_stats returns (hyperbolic_ops.py:437-439)."""
    if ev is None:
        return None
    out = dict(zip(EVOLUTION_KEYS, ev["vec"].tolist()))
    out["anchor_beta"] = ev["anchor_beta"]
    out["epsilon"] = ev["epsilon"]
    return out


def embedding_stats(radius, c):
    """HyperbolicOps.log_embedding_stats (hyperbolic_ops.py:235-269) on the device from the row
    norms `radius` (get_radius: |x| clamped at 1e-6): [mean, max, min, std, pct near boundary]."""
    max_radius = 1.0 / (float(c) ** 0.5)
    return torch.stack([radius.mean(), radius.max(), radius.min(), radius.std(),
                        (radius > 0.9 * max_radius).float().mean() * 100]).detach()


def embedding_dict(vec, name, c):
    mean, mx, mn, std, pct = vec.tolist()
    return {"name": name, "mean_norm": mean, "max_norm": mx, "min_norm": mn, "std_norm": std,
            "max_allowed": 1.0 / (float(c) ** 0.5), "pct_near_boundary": pct}


def log_embedding(model, h, name, c):
    """hyperbolic_model.py:791-792 / :932-933: the stats of `h` kept on the device in
    model.embedding_stats[name]; the debug line only when DEBUG is enabled."""
    from .hyperbolic_ops import HyperbolicOps
    vec = embedding_stats(HyperbolicOps.get_radius(h.detach()), c)
    model.__dict__.setdefault("embedding_stats", {})[name] = vec
    if logger.isEnabledFor(logging.DEBUG):
        s = embedding_dict(vec, name, c)
        logger.debug("%s stats: mean=%.4f, max=%.4f, near_boundary=%.2f%%", name, s["mean_norm"], s["max_norm"],
                     s["pct_near_boundary"])
    return vec


def log_timestep(i, gate_mean, ev):
    """The per-timestep debug lines of hyperbolic_model.py:856, :872-882."""
    if not logger.isEnabledFor(logging.DEBUG):
        return
    logger.debug("Time step %d: time_gate_mean=%.4f", i, float(gate_mean))
    s = evolution_dict(ev)
    if s:
        logger.debug("Time step %d: radius_delta_mean=%.4f, radius_delta_std=%.4f, dynamic_radius_mean=%.4f, "
                     "static_radius_mean=%.4f, base_radius_mean=%.4f, anchor_beta=%.4f", i, s["delta_mean"],
                     s["delta_std"], s["dynamic_radius_mean"], s["static_radius_mean"], s["base_radius_mean"],
                     s["anchor_beta"])


def record_losses(model, le, lr, ls, lrad):
    """hyperbolic_model.py:1076-1086: one loss-components entry per get_loss (per mini-batch)."""
    model.training_stats.raw("loss_components").append(
        {"loss_ent": le.detach().reshape(()), "loss_rel": lr.detach().reshape(()),
         "loss_static": ls.detach().sum().reshape(()), "loss_radius": lrad.detach().reshape(())})
    if logger.isEnabledFor(logging.DEBUG):
        logger.debug("Loss components: ent=%.4f, rel=%.4f, static=%.4f, radius=%.4f", float(le), float(lr),
                     float(ls.sum()), float(lrad))


def gradient_stats(model):
    """hyperbolic_model.py:1090-1108: the total gradient norm over all parameters, appended to
    training_stats["gradient_norms"] as a device scalar (and returned as one); the per-parameter
    norms above 1 are listed in a debug line when DEBUG is enabled."""
    named = [(n, p.grad) for n, p in model.named_parameters() if p.grad is not None]
    if not named:
        total = torch.zeros((), device=next(model.parameters()).device)
    else:
        norms = torch._foreach_norm([g for _, g in named])
        total = torch.stack(norms).double().pow(2).sum().sqrt().float()
        if logger.isEnabledFor(logging.DEBUG):
            host = torch.stack(norms).tolist()
            logger.debug("Total gradient norm: %.4f", float(total))
            big = {n: v for (n, _), v in zip(named, host) if v > 1.0}
            if big:
                logger.debug("Large gradients: %s", big)
    model.training_stats.raw("gradient_norms").append(total)
    return total


def training_summary(model):
    """hyperbolic_model.py:1110-1127."""
    summary = {"curvature": float(model.get_curvature())}
    ev = model.temporal_radius_evolution.get_evolution_stats()
    if ev:
        summary["radius_delta_mean"] = ev.get("delta_mean")
        summary["radius_delta_std"] = ev.get("delta_std")
        summary["dynamic_radius_mean"] = ev.get("dynamic_radius_mean")
        summary["static_radius_mean"] = ev.get("static_radius_mean")
        summary["base_radius_mean"] = ev.get("base_radius_mean")
        summary["anchor_beta"] = ev.get("anchor_beta", model.radius_anchor_beta)
    gates = model.training_stats.raw("time_gate_values")
    if len(gates):
        summary["avg_time_gate"] = float(torch.as_tensor(gates).mean()) if not torch.is_tensor(gates) \
            else float(gates.double().mean())
    return summary
