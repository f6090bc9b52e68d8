"""Privacy accounting for DP-SGD: the Renyi-DP accountant of the sampled
Gaussian mechanism and the noise-multiplier search that opacus's
`PrivacyEngine.make_private_with_epsilon` runs (main_0430.py:152-162, base_train.py:337-348).

opacus is not installed here (and not pinned by the reference), so this restates the published
algorithm it implements:
  * RDP of the Poisson-subsampled Gaussian mechanism, Mironov, Talwar & Zhang, "Renyi Differential
    Privacy of the Sampled Gaussian Mechanism" (2019), Sec. 3.3: integer orders by the binomial
    expansion, fractional orders by the two-sided series with erfc tails (opacus
    accountants/analysis/rdp.py, itself the TensorFlow-Privacy rdp_accountant);
  * RDP -> (eps, delta) with the conversion of Balle et al. 2020 (Thm. 21):
      eps = rdp - (log delta + log a) / (a - 1) + log((a - 1) / a), minimised over the orders;
  * get_noise_multiplier: double sigma from 10 until eps(sigma) < target, then bisect until
    target - eps <= epsilon_tolerance (0.01), returning the upper end (opacus accountants/utils.py).
opacus >= 1.3 defaults `PrivacyEngine(accountant="prv")`; the PRV accountant is not restated here —
`accountant="rdp"` (opacus's other built-in) is what this module computes, and the build says so.
Pinned by closed forms (q = 1: rdp = a / (2 sigma^2)) and by the published TensorFlow-Privacy test
vectors (tests/test_privacy_cpu.py); opacus itself is absent: parity with it is unpinned.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import special

DEFAULT_ALPHAS = [1 + x / 10.0 for x in range(1, 100)] + list(range(12, 64))
MAX_SIGMA = 1e6


def _log_add(logx: float, logy: float) -> float:
    a, b = min(logx, logy), max(logx, logy)
    if a == -np.inf:
        return b
    return math.log1p(math.exp(a - b)) + b


def _log_sub(logx: float, logy: float) -> float:
    if logx < logy:
        raise ValueError("the result of subtraction must be non-negative")
    if logy == -np.inf:
        return logx
    if logx == logy:
        return -np.inf
    try:
        return math.log(math.expm1(logx - logy)) + logy
    except OverflowError:
        return logx


def _log_erfc(x: float) -> float:
    return math.log(2) + special.log_ndtr(-x * 2 ** 0.5)


def _log_a_int(q: float, sigma: float, alpha: int) -> float:
    log_a = -np.inf
    for i in range(alpha + 1):
        log_coef_i = math.log(special.binom(alpha, i)) + i * math.log(q) + (alpha - i) * math.log(1 - q)
        log_a = _log_add(log_a, log_coef_i + (i * i - i) / (2 * sigma ** 2))
    return float(log_a)


def _log_a_frac(q: float, sigma: float, alpha: float) -> float:
    log_a0, log_a1 = -np.inf, -np.inf
    i = 0
    z0 = sigma ** 2 * math.log(1 / q - 1) + 0.5
    while True:
        coef = special.binom(alpha, i)
        log_coef = math.log(abs(coef))
        j = alpha - i
        log_t0 = log_coef + i * math.log(q) + j * math.log(1 - q)
        log_t1 = log_coef + j * math.log(q) + i * math.log(1 - q)
        log_e0 = math.log(0.5) + _log_erfc((i - z0) / (math.sqrt(2) * sigma))
        log_e1 = math.log(0.5) + _log_erfc((z0 - j) / (math.sqrt(2) * sigma))
        log_s0 = log_t0 + (i * i - i) / (2 * sigma ** 2) + log_e0
        log_s1 = log_t1 + (j * j - j) / (2 * sigma ** 2) + log_e1
        if coef > 0:
            log_a0 = _log_add(log_a0, log_s0)
            log_a1 = _log_add(log_a1, log_s1)
        else:
            log_a0 = _log_sub(log_a0, log_s0)
            log_a1 = _log_sub(log_a1, log_s1)
        i += 1
        if max(log_s0, log_s1) < -30:
            break
    return _log_add(log_a0, log_a1)


def _rdp_one(q: float, sigma: float, alpha: float) -> float:
    if q == 0:
        return 0.0
    if sigma == 0:
        return np.inf
    if q == 1.0:
        return alpha / (2 * sigma ** 2)
    if np.isinf(alpha):
        return np.inf
    log_a = _log_a_int(q, sigma, int(alpha)) if float(alpha).is_integer() else _log_a_frac(q, sigma, alpha)
    return log_a / (alpha - 1)


def compute_rdp(*, q: float, noise_multiplier: float, steps: int, orders) -> np.ndarray | float:
    """RDP of `steps` compositions of the sampled Gaussian mechanism at each order."""
    if isinstance(orders, (int, float)):
        return _rdp_one(q, noise_multiplier, orders) * steps
    return np.array([_rdp_one(q, noise_multiplier, a) for a in orders]) * steps


def get_privacy_spent(*, orders, rdp, delta: float) -> tuple[float, float]:
    """(eps, best order) for the given RDP curve and delta (Balle et al. 2020 conversion)."""
    orders_vec = np.atleast_1d(orders).astype(np.float64)
    rdp_vec = np.atleast_1d(rdp).astype(np.float64)
    if len(orders_vec) != len(rdp_vec):
        raise ValueError("orders and rdp must have the same length")
    with np.errstate(invalid="ignore", divide="ignore"):
        eps = rdp_vec - (np.log(delta) + np.log(orders_vec)) / (orders_vec - 1) + np.log((orders_vec - 1) / orders_vec)
    if np.isnan(eps).all():
        return np.inf, np.nan
    i = int(np.nanargmin(eps))
    return float(eps[i]), float(orders_vec[i])


class RDPAccountant:
    """opacus RDPAccountant: history of (noise_multiplier, sample_rate, steps) segments."""

    def __init__(self):
        self.history: list[tuple[float, float, int]] = []

    def step(self, *, noise_multiplier: float, sample_rate: float) -> None:
        if self.history and self.history[-1][:2] == (noise_multiplier, sample_rate):
            nm, sr, n = self.history.pop()
            self.history.append((nm, sr, n + 1))
        else:
            self.history.append((noise_multiplier, sample_rate, 1))

    def get_privacy_spent(self, *, delta: float, alphas=None) -> tuple[float, float]:
        if not self.history:
            return 0.0, 0.0
        alphas = DEFAULT_ALPHAS if alphas is None else alphas
        rdp = sum(compute_rdp(q=sr, noise_multiplier=nm, steps=n, orders=alphas) for nm, sr, n in self.history)
        return get_privacy_spent(orders=alphas, rdp=rdp, delta=delta)

    def get_epsilon(self, delta: float, alphas=None) -> float:
        return self.get_privacy_spent(delta=delta, alphas=alphas)[0]

    def __len__(self):
        return len(self.history)

    @staticmethod
    def mechanism() -> str:
        return "rdp"


def create_accountant(mechanism: str):
    if mechanism == "rdp":
        return RDPAccountant()
    raise NotImplementedError(f"accountant {mechanism!r}: only the RDP accountant is restated here "
                              "(opacus's default 'prv' is not; pass accountant='rdp')")


def get_noise_multiplier(*, target_epsilon: float, target_delta: float, sample_rate: float, epochs: int | None = None,
                         steps: int | None = None, accountant: str = "rdp", epsilon_tolerance: float = 0.01,
                         **kwargs) -> float:
    """Smallest noise multiplier (within epsilon_tolerance) whose eps after `steps` (or
    epochs / sample_rate) steps is below target_epsilon."""
    if (steps is None) == (epochs is None):
        raise ValueError("get_noise_multiplier takes as input EITHER a number of steps or a number of epochs")
    if steps is None:
        steps = int(epochs / sample_rate)
    eps_high = float("inf")
    acc = create_accountant(accountant)
    sigma_low, sigma_high = 0.0, 10.0
    while eps_high > target_epsilon:
        sigma_high = 2 * sigma_high
        acc.history = [(sigma_high, sample_rate, steps)]
        eps_high = acc.get_epsilon(delta=target_delta, **kwargs)
        if sigma_high > MAX_SIGMA:
            raise ValueError("The privacy budget is too low.")
    while target_epsilon - eps_high > epsilon_tolerance:
        sigma = (sigma_low + sigma_high) / 2
        acc.history = [(sigma, sample_rate, steps)]
        eps = acc.get_epsilon(delta=target_delta, **kwargs)
        if eps < target_epsilon:
            sigma_high, eps_high = sigma, eps
        else:
            sigma_low = sigma
    return sigma_high
