"""Parity helpers: GPU (product) vs oracle (CPU restatement).

Tolerance (BASELINE.json north_star): per-channel |d| <= 1e-4 on pixels whose
discrete decisions agree; pixels beyond it are counted as decision mismatches
(silhouettes / shadow edges) and must stay below a small fraction.
"""
import numpy as np

TOL = 1e-4


def compare(rgb_a, argb_a, rgb_b, argb_b, tol=TOL):
    d = np.abs(rgb_a.astype(np.float64) - rgb_b.astype(np.float64)).max(-1)
    bad = d > tol
    good = ~bad
    argb_mis = int(((argb_a != argb_b) & good).sum())
    return {
        "pixels": int(d.size),
        "max_abs": float(d.max()) if d.size else 0.0,
        "mismatch": int(bad.sum()),
        "mismatch_frac": float(bad.mean()) if d.size else 0.0,
        "argb_mismatch_on_good": argb_mis,
        "argb_equal": int((argb_a == argb_b).sum()),
    }


def assert_exact_decisions(c):
    """Every pixel within the per-channel tolerance (no decision mismatch: hit object, shadow,
    TIR, photon k-set all agree) and every such pixel's ARGB int equal -- what was observed on
    every deterministic-decision config."""
    assert c["mismatch"] == 0, c
    assert c["argb_mismatch_on_good"] == 0, c
