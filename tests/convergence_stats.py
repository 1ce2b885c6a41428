"""Per-epoch bound for a run that is another DRAW of the reference's training (device dropout, bf16).

Shared by tests/test_gpu_convergence.py (the check) and tests/test_convergence_calibration_cpu.py
(its false-alarm rate on the reference's own draws).  At every epoch and metric the mean of D draws
may differ from the mean of the reference's draws by at most

    max(0.5 pp, K_SIGMA * sigma_e * sqrt(1/D + 1/R), 2 samples of the metric's denominator)

with sigma_e the reference draws' standard deviation at that epoch (R draws), floored at
SIGMA_FLOOR: a metric that all reference draws hit exactly (100 % at a saturated epoch) has
sample sigma 0, not population sigma 0.  Many epoch-metric cells are compared per run and a run's
epochs are correlated (a draw that learns the poisoned subset early stays ahead), so the rule allows
at most MAX_CELLS cells past the bound and none past MAX_RATIO times it; calibrated on the reference's
own draws (tests/test_convergence_calibration_cpu.py: 0 of 420 leave-3-out splits fail it, against
4 of 420 for "at most one cell")."""
import numpy as np

K_SIGMA = 4.0
# per-config multiplier where the calibration allows a tighter one (tests/test_convergence_calibration_cpu.py
# measures its false-alarm rate on the reference's own draws at this value)
K_BY_CFG = {"flowmur": 3.5}
SIGMA_FLOOR = 0.5
MAX_CELLS = 2
MAX_RATIO = 2.0


def k_sigma(name, n_dev=None):
    return K_BY_CFG.get(name, K_SIGMA)

# (label, source, column, denominator key): test() tuple (clean acc, ASR, clean loss, bd loss),
# train() tuple (loss, mix acc, ASR)
METRICS = (("test clean acc", "te", 0, "n_test"), ("test ASR", "te", 1, "n_bd"),
           ("train acc", "tr", 1, "n_train"), ("train ASR", "tr", 2, "n_pois"))


def ref_draws(conv_ref, name):
    """(R, E, 4) test() tuples and (R, E, 3) train() tuples: the fixture run + its RNG replicates."""
    te = np.concatenate([conv_ref[f"{name}_test"][None], conv_ref[f"{name}_test_seeds_ep"]])
    tr = np.concatenate([conv_ref[f"{name}_train"][None], conv_ref[f"{name}_train_seeds_ep"]])
    return te, tr


def draw_bound(ref_vals, n_dev, n_den, k_sigma=K_SIGMA):
    """ref_vals (R, E): allowed |mean of n_dev draws - mean of ref_vals| per epoch (pp)."""
    sig = np.maximum(ref_vals.std(axis=0, ddof=1), SIGMA_FLOOR)
    se = sig * np.sqrt(1.0 / n_dev + 1.0 / ref_vals.shape[0])
    return np.maximum(np.maximum(0.5, k_sigma * se), 200.0 / n_den)


def violations(ours_te, ours_tr, ref_te, ref_tr, dens, k_sigma=K_SIGMA):
    """[(metric, epoch, ours, ref mean, bound)] outside the bound; ours_* (D, E, ...)."""
    bad = []
    srcs = {"te": (ours_te, ref_te), "tr": (ours_tr, ref_tr)}
    for what, src, col, den in METRICS:
        o, r = srcs[src][0][:, :, col], srcs[src][1][:, :, col]
        bound = draw_bound(r, o.shape[0], dens[den], k_sigma)
        gap = np.abs(o.mean(0) - r.mean(0))
        for e in np.nonzero(gap > bound)[0]:
            bad.append((what, int(e) + 1, float(o[:, e].mean()), float(r[:, e].mean()), float(bound[e])))
    return bad


def rule_fails(bad):
    """True when the violations list breaks the per-run rule (MAX_CELLS, MAX_RATIO)."""
    return len(bad) > MAX_CELLS or any(abs(b[2] - b[3]) > MAX_RATIO * b[4] for b in bad)


def detectable_shift(ref_vals, n_dev, n_den, k_sigma=K_SIGMA, power=0.9, trials=4000, seed=0, step=0.25):
    """Smallest systematic shift (pp, applied at every epoch of ONE metric, downward and clipped at
    0) that the per-run rule flags in at least `power` of simulated runs: the difference of the two
    means (n_dev draws, R reference draws) is modelled as N(-shift, S (1/n_dev + 1/R)) over the
    epochs, S the reference draws' covariance ACROSS epochs (a draw ahead at one epoch stays ahead:
    independent per-epoch noise would overstate the power), against draw_bound.  One metric's
    cells alone: no other metric contributes violations, so this is what the rule resolves on it."""
    rng = np.random.default_rng(seed)
    R = ref_vals.shape[0]
    mu = ref_vals.mean(0)
    bound = draw_bound(ref_vals, n_dev, n_den, k_sigma)
    cov = np.cov(ref_vals, rowvar=False, ddof=1) * (1.0 / n_dev + 1.0 / R)
    noise = rng.multivariate_normal(np.zeros(mu.size), cov, size=trials, method="eigh")
    d = 0.0
    while d < 100.0:
        ours = np.maximum(mu - d + noise, 0.0)
        gap = np.abs(ours - mu)
        over = gap > bound
        fails = (over.sum(1) > MAX_CELLS) | (gap > MAX_RATIO * bound).any(1)
        if fails.mean() >= power:
            return d
        d += step
    return float("inf")
