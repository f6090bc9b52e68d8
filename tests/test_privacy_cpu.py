"""RDP accountant + noise-multiplier search (eegfusion/privacy.py) — opacus is absent, so the
restatement is pinned by closed forms and by the published TensorFlow-Privacy rdp_accountant test
vectors (the algorithm opacus's accountants/analysis/rdp.py carries over); parity with opacus's
own runs is unpinned."""
import math

import numpy as np
import pytest

from eegfusion.privacy import (DEFAULT_ALPHAS, RDPAccountant, compute_rdp, create_accountant, get_noise_multiplier,
                               get_privacy_spent)


def test_rdp_scalar_tf_privacy_vector():
    # rdp_accountant_test.test_compute_rdp_scalar: q=0.1, sigma=2, 10 steps, order 5
    assert compute_rdp(q=0.1, noise_multiplier=2, steps=10, orders=5) == pytest.approx(0.07737, abs=5e-6)


def test_rdp_sequence_tf_privacy_vector():
    # rdp_accountant_test.test_compute_rdp_sequence (fractional and integer orders, inf)
    r = compute_rdp(q=0.01, noise_multiplier=2.5, steps=50, orders=[1.5, 2.5, 5, 50, 100, np.inf])
    ref = [6.5007e-04, 1.0854e-03, 2.1808e-03, 2.3846e-02, 1.6742e+02, np.inf]
    np.testing.assert_allclose(r, ref, rtol=1e-4)


def test_eps_tf_privacy_vector_classic_conversion():
    # rdp_accountant_test.test_get_privacy_spent_check_target_delta (q=0.01, sigma=4, 10000 steps,
    # orders 2..32, delta 1e-5: eps 1.258575 at order 20) under the classic conversion
    # eps = rdp - log(delta)/(a-1); opacus uses the tighter Balle et al. 2020 form, checked below to
    # be <= it at every order
    orders = np.arange(2, 33)
    rdp = compute_rdp(q=0.01, noise_multiplier=4, steps=10000, orders=orders)
    classic = rdp - math.log(1e-5) / (orders - 1)
    i = int(np.argmin(classic))
    assert classic[i] == pytest.approx(1.258575, abs=1e-5) and orders[i] == 20
    eps, _ = get_privacy_spent(orders=orders, rdp=rdp, delta=1e-5)
    assert eps < classic[i]


def test_full_sampling_closed_form():
    # q = 1: the Gaussian mechanism, RDP(a) = a / (2 sigma^2) per step
    for a in (1.5, 2.0, 7.0, 33.0):
        assert compute_rdp(q=1.0, noise_multiplier=1.3, steps=3, orders=a) == pytest.approx(3 * a / (2 * 1.3 ** 2))
    assert compute_rdp(q=0.0, noise_multiplier=1.0, steps=5, orders=3.0) == 0.0


def test_accountant_history_and_monotonicity():
    acc = RDPAccountant()
    assert acc.get_epsilon(1e-5) == 0.0
    for _ in range(100):
        acc.step(noise_multiplier=1.1, sample_rate=0.01)
    assert acc.history == [(1.1, 0.01, 100)]
    e100 = acc.get_epsilon(1e-5)
    for _ in range(100):
        acc.step(noise_multiplier=1.1, sample_rate=0.01)
    assert acc.get_epsilon(1e-5) > e100 > 0
    with pytest.raises(NotImplementedError):
        create_accountant("prv")


@pytest.mark.parametrize("eps,q,epochs", [(1.0, 1 / 300, 30), (3.0, 1 / 301, 50), (0.5, 8 / 2402, 10)])
def test_noise_multiplier_search(eps, q, epochs):
    sigma = get_noise_multiplier(target_epsilon=eps, target_delta=q, sample_rate=q, epochs=epochs)
    steps = int(epochs / q)
    rdp = compute_rdp(q=q, noise_multiplier=sigma, steps=steps, orders=DEFAULT_ALPHAS)
    got, _ = get_privacy_spent(orders=DEFAULT_ALPHAS, rdp=rdp, delta=q)
    assert got <= eps and eps - got <= 0.01 + 1e-9             # within opacus's epsilon_tolerance
    # a noticeably smaller sigma overspends the budget
    rdp2 = compute_rdp(q=q, noise_multiplier=sigma * 0.97, steps=steps, orders=DEFAULT_ALPHAS)
    assert get_privacy_spent(orders=DEFAULT_ALPHAS, rdp=rdp2, delta=q)[0] > got
