"""Error of the short sigmoid / tanh forms of decoder_persist.hip (sigm_f, tanh_f) against float64,
with float32 arithmetic emulated in numpy. v_exp_f32 and v_rcp_f32 are modelled as the exact
result rounded to float32 and then perturbed by one ulp (their documented accuracy), so the bound
printed is a worst case over both rounding directions.

  python tools/fast_math_err.py
"""
import numpy as np

f32 = np.float32


def ulp_perturb(v, sign):
    return np.nextafter(v, np.where(sign > 0, np.float32(np.inf), np.float32(-np.inf))).astype(f32)


def exp2_hw(x, s):
    return ulp_perturb(np.exp2(x.astype(np.float64)).astype(f32), s)


def rcp_hw(x, s):
    return ulp_perturb((1.0 / x.astype(np.float64)).astype(f32), s)


def sigm_f(x, s):
    return rcp_hw(f32(1) + exp2_hw(f32(-1.4426950408889634) * x, s), -s)


def tanh_f(x, s):
    ax = np.abs(x).astype(f32)
    e = exp2_hw(f32(-2.8853900817779268) * ax, s)
    big = ((f32(1) - e) * rcp_hw(f32(1) + e, -s)).astype(f32)
    x2 = (ax * ax).astype(f32)
    poly = (x2 * f32(0.021869488) + f32(-0.053968254)).astype(f32)
    poly = (x2 * poly + f32(0.13333334)).astype(f32)
    poly = (x2 * poly + f32(-0.33333334)).astype(f32)
    small = ((ax * x2).astype(f32) * poly + ax).astype(f32)
    return np.copysign(np.where(ax < f32(0.25), small, big), x).astype(f32)


def tanh_e(x, s):  # the attention energies' form: no small-argument polynomial
    ax = np.abs(x).astype(f32)
    e = exp2_hw(f32(-2.8853900817779268) * ax, s)
    return np.copysign(((f32(1) - e) * rcp_hw(f32(1) + e, -s)).astype(f32), x).astype(f32)


def main():
    x = np.concatenate([np.linspace(-30, 30, 2_000_001), np.linspace(-0.3, 0.3, 600_001)]).astype(f32)
    xd = x.astype(np.float64)
    for name, fn, ref in (("sigm_f", sigm_f, 1 / (1 + np.exp(-xd))), ("tanh_f", tanh_f, np.tanh(xd)),
                          ("tanh_e", tanh_e, np.tanh(xd))):
        err = max(np.abs(fn(x, s).astype(np.float64) - ref).max() for s in (-1, 1))
        libm = np.abs((1 / (1 + np.exp(-x)) if name == "sigm_f" else np.tanh(x)).astype(np.float64) - ref).max()
        print(f"{name}: max |error| {err:.2e} (numpy float32 libm: {libm:.2e})")


if __name__ == "__main__":
    main()
