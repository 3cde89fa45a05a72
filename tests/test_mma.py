"""MMA optimiser (tclb_amd.utils.mma; NLopt MMA is the reference Optimize default)."""
import numpy as np

from tclb_amd.utils.mma import mma_minimize


def test_bound_constrained_quadratic():
    target = np.array([0.3, -0.7, 2.5, 0.1])
    r = mma_minimize(lambda x: (float(np.sum((x - target) ** 2)), 2 * (x - target)), np.zeros(4),
                     -np.ones(4), np.ones(4), maxeval=200, ftol_abs=1e-12)
    np.testing.assert_allclose(r.x, np.clip(target, -1, 1), atol=1e-5)
    assert all(b <= a + 1e-9 for a, b in zip(r.history, r.history[1:]))    # monotone (conservative)
    assert r.evaluations < 60


def test_rosenbrock():
    def f(x):
        a, b = x
        return (1 - a) ** 2 + 100 * (b - a * a) ** 2, np.array([-2 * (1 - a) - 400 * a * (b - a * a),
                                                                200 * (b - a * a)])
    r = mma_minimize(f, np.array([-1.2, 1.0]), np.array([-2.0, -2.0]), np.array([2.0, 2.0]), maxeval=3000,
                     ftol_abs=1e-16)
    np.testing.assert_allclose(r.x, [1, 1], atol=1e-2)   # MMA creeps along curved valleys


def test_inequality_constraint_is_active():
    # min sum (x-1)^2  s.t.  sum x <= 2  ->  x = 0.5
    r = mma_minimize(lambda x: (float(np.sum((x - 1) ** 2)), 2 * (x - 1)), np.zeros(4), np.zeros(4), np.ones(4) * 3,
                     constraints=[lambda x: (float(np.sum(x) - 2), np.ones(4))], maxeval=300, ftol_abs=1e-14)
    np.testing.assert_allclose(r.x, 0.5, atol=1e-4)
