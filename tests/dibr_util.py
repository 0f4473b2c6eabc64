"""Test helpers for the compact DIB-R soft-mask state (softtile.hip layout, include/kaolin_hip.h).

oracle.decode_compact() turns the records back into the reference's (B,H,W,K) slot tensors, so
the oracle's backward can be driven with the GPU forward's own saved values: the backward parity
is then checked on identical inputs (the forward's probabilities are checked on their own, to
expf ulps -- the GPU's expf and glibc's differ by an ulp now and then)."""
import numpy as np

from oracle.oracle import decode_compact  # noqa: F401


def assert_grads_equal(got, ref):
    """DIB-R gradients: the reference's float per-pixel / per-hit terms summed in double and
    rounded once, on the GPU (any order of lanes / atomics) and in the oracle (pixel order).
    Float terms whose magnitudes span less than ~2^29 sum exactly in double, so both are the
    correctly rounded sum and equal bit for bit; where one face's terms span more (a
    probability near 0 beside one near 1), the two double sums may differ in their last bits
    and the rounded results by one ulp -- allowed for at most 1 element in 10^4.  NaN where
    the oracle has NaN.  (f64 terms do not sum exactly in double: there the two orders agree
    to ~1e-15 relative.)"""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape and got.dtype == ref.dtype
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = np.isfinite(ref)
    if got.dtype == np.float64:
        scale = max(1.0, float(np.abs(ref[fin]).max())) if fin.any() else 1.0
        np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-12, atol=1e-12 * scale)
        return
    np.testing.assert_array_equal(got[~fin], ref[~fin])
    diff = got[fin] != ref[fin]
    assert diff.sum() <= max(1, diff.size // 10000), f'{int(diff.sum())} of {diff.size} elements differ'
    np.testing.assert_array_max_ulp(got[fin], ref[fin], maxulp=1)


def state_arrays(state):
    """The compact state's tensors as numpy arrays (hits, rec_face, rec_prob)."""
    return (state.hits.detach().cpu().numpy(), state.rec_face.detach().cpu().numpy(),
            state.rec_prob.detach().cpu().numpy())


# ---- the dev library (make dev: kaolin/_lib/dev/libkaolin_hip.so, KL_DEV=1).  The product library
# has no dev controls; tests marked `devlib` switch between the product path and a measured
# alternative, or force a fallback, through them.  They run in tests/test_gpu_devlib.py's child
# process against the dev build; in a process on the product library they skip the parts that
# need it (setting a control back to its default, 0, is a no-op there).
def dev_lib():
    """The loaded library's ctypes handle if it is the dev build, else None."""
    import ctypes
    from kaolin import _native as N
    lib = N.lib()
    if not hasattr(lib, 'kl_dev_build'):
        return None
    lib.kl_dev_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.kl_dev_set_flags.argtypes = [ctypes.c_int]
    lib.kl_dev_get_stat.argtypes = [ctypes.c_int]
    lib.kl_dev_get_stat.restype = ctypes.c_int
    return lib


def require_dev():
    import pytest
    lib = dev_lib()
    if lib is None:
        pytest.skip('needs the dev library (make dev): run by tests/test_gpu_devlib.py')
    return lib


def dev_param(idx, val):
    """kl_dev_set_param on the dev library; 0 (the default) is a no-op on the product library."""
    lib = dev_lib()
    if lib is None:
        if val == 0:
            return
        require_dev()
    lib.kl_dev_set_param(idx, val)


def dev_flags(flags):
    lib = dev_lib()
    if lib is None:
        if flags == 0:
            return
        require_dev()
    lib.kl_dev_set_flags(flags)
