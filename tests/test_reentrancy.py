"""Reentrancy of the C ABI ("the JNI layer must be
reentrant").  In the reference, Spark's N executor task threads call the primitives
concurrently in one JVM (S/TimeSeriesRDD.scala:417-421, local[N]); here N Python threads call
the library concurrently through ctypes (which releases the GIL for the foreign call):

* device entry points on the NULL stream (hipStreamPerThread of each thread) and the `_host`
  entry points (borrowed staging slot sets), on different panels at once -- every result
  bit-identical to the same call made single-threaded;
* sts_last_error() stays per thread while other threads fail and succeed;
* staging memory stays bounded: short-lived threads never grow the slot-set pool past its
  limit, device memory stays flat, sts_staging_release() frees the idle sets, and a failing
  call followed by a smaller one on the same thread gives exact results.
GPU only (the CPU side of the same properties: tests/test_sanitizers.py, ThreadSanitizer).
"""
import ctypes
import threading

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

NTHREADS = 8


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    from sparkts import _native
    _native.ensure_device(0)
    return _t


def lib():
    from sparkts import _native
    return _native.lib()


def P(a):
    return a.ctypes.data


def bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and bool(((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))).all())


def pool_info():
    v = np.zeros(8, dtype=np.int64)
    assert lib().sts_staging_pool_info(P(v)) == 0
    return dict(zip(["live", "idle", "borrowed", "limit", "high", "lost", "waits", "set_bytes"], v.tolist()))


def run_threads(fns):
    """Run each fn in its own thread (all started together); re-raise the first failure."""
    from sparkts import _native
    errs = [None] * len(fns)
    out = [None] * len(fns)
    barrier = threading.Barrier(len(fns))

    def body(i):
        try:
            _native.ensure_device(0)            # sts_init per thread (selects the device)
            barrier.wait()
            out[i] = fns[i]()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs[i] = e
    th = [threading.Thread(target=body, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    for e in errs:
        if e is not None:
            raise e
    return out


# ---- the three kinds of calls, one panel each ----

def call_fill_autocorr_device(torch, x, K=20):
    """sts_fill_autocorr on HBM data, NULL stream (the calling thread's per-thread stream)."""
    S, T = x.shape
    xd = torch.as_tensor(x, device="cuda:0")
    fd = torch.empty_like(xd)
    ad = torch.empty((S, K), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()                    # the upload is on torch's stream
    st = lib().sts_fill_autocorr(xd.data_ptr(), fd.data_ptr(), S, T, T, T, 0, K, ad.data_ptr(), None, None)
    assert st == 0, lib().sts_last_error()
    assert lib().sts_stream_synchronize(None) == 0
    return fd.cpu().numpy(), ad.cpu().numpy()


def call_fill_diff_ewma_host(x):
    S, T = x.shape
    out = np.empty_like(x)
    sm = np.full(S, 0.3)
    err = np.zeros(S, dtype=np.int32)
    st = lib().sts_fill_diff_ewma_host(P(x), P(out), S, T, T, 3, 1, P(sm), P(err))
    assert st == 0, lib().sts_last_error()
    return out, err


def call_ar_fit_remove_host(x, p=5):
    S, T = x.shape
    out = np.empty_like(x)
    c = np.empty(S)
    coef = np.empty((S, p))
    err = np.zeros(S, dtype=np.int32)
    st = lib().sts_ar_fit_remove_host(P(x), P(out), S, T, T, p, 0, P(c), P(coef), P(err))
    assert st == 0, lib().sts_last_error()
    return out, c, coef, err


def panels(seed):
    """Per-thread inputs: ~40-70 MB host panels (the _host calls run several chunks)."""
    rng = np.random.default_rng(seed)
    S = int(rng.integers(18000, 26000))
    a = oracle.gen_panel(seed, S, 390, 0.05)
    b = oracle.gen_ar_panel(seed, int(rng.integers(1500, 3000)), 2520, 5)
    d = oracle.gen_panel(seed + 100, int(rng.integers(300, 600)), 2520, 0.05)
    return a, b, d


def test_concurrent_calls_are_bit_exact(torch):
    work = [panels(1000 + i) for i in range(NTHREADS)]

    def job(i):
        a, b, d = work[i]
        kind = i % 3
        if kind == 0:
            return call_fill_autocorr_device(torch, d)
        if kind == 1:
            return call_fill_diff_ewma_host(a)
        return call_ar_fit_remove_host(b)

    # reference: the same calls one after another on this thread
    ref = [job(i) for i in range(NTHREADS)]
    for rep in range(2):
        got = run_threads([(lambda i=i: job(i)) for i in range(NTHREADS)])
        for i in range(NTHREADS):
            for g, r in zip(got[i], ref[i]):
                assert bits(np.asarray(g, dtype=np.float64), np.asarray(r, dtype=np.float64)), \
                    "thread %d (kind %d) differs from the single-threaded call (rep %d)" % (i, i % 3, rep)
    # and the single-threaded results are the oracle's (spot check, one panel per kind)
    a, b, d = work[1]
    rf = oracle.panel_fill_diff_ewma(a[:200], 0.3, threads=4)
    assert bits(ref[1][0][:200], rf)
    info = pool_info()
    assert info["borrowed"] == 0 and info["live"] <= info["limit"]


def test_last_error_is_per_thread(torch):
    nan_panel = np.full((4, 50), np.nan)

    def job(i):
        msgs = []
        for k in range(20):
            if (i + k) % 2:
                # a failing call with a message unique to this thread
                st = lib().sts_fill_host(P(nan_panel), P(np.empty_like(nan_panel)), -(i + 1), 50, 50, 0, None)
                assert st != 0
                msgs.append(("S=%d," % -(i + 1), lib().sts_last_error().decode()))
            else:
                out = np.empty_like(nan_panel)
                err = np.zeros(4, dtype=np.int32)
                assert lib().sts_fill_host(P(nan_panel), P(out), 4, 50, 50, 1, P(err)) == 0   # nearest: per-series errors
                assert (err != 0).all()
        return msgs

    for msgs in run_threads([(lambda i=i: job(i)) for i in range(NTHREADS)]):
        for want, got in msgs:
            assert want in got, (want, got)


def test_staging_memory_is_bounded_across_short_lived_threads(torch):
    from sparkts import _native
    x = oracle.gen_panel(7, 30000, 390, 0.05)         # 94 MB: several chunks per call
    ref = call_fill_diff_ewma_host(x)
    assert lib().sts_staging_set_limit(2) == 0
    try:
        lib().sts_staging_release()
        torch.cuda.synchronize()
        free0 = None
        for wave in range(6):                           # 6 x 8 threads that call once and exit
            got = run_threads([(lambda: call_fill_diff_ewma_host(x)) for _ in range(NTHREADS)])
            for g in got:
                assert bits(g[0], ref[0])
            info = pool_info()
            assert info["live"] <= 2 and info["high"] <= 4 and info["borrowed"] == 0, info
            free = torch.cuda.mem_get_info()[0]
            if wave == 0:
                free0 = free
            else:   # flat after the first wave: no per-thread buffers survive their threads
                assert abs(free - free0) < (64 << 20), (wave, free0, free)
        assert pool_info()["waits"] > 0                 # 8 callers, 2 sets: they took turns
        assert lib().sts_staging_release() == 0
        assert pool_info()["live"] == 0
    finally:
        _native.lib().sts_staging_set_limit(4)


def test_failing_call_then_smaller_call_same_thread(torch):
    """a call that fails (here: per-series errors turned into the return status,
    decided after every chunk) followed by a smaller call on the same thread -- no stale chunk
    may land in the second call's outputs."""
    S, T = 3000, 2520
    x = oracle.gen_ar_panel(11, S, T, 5)
    x[S - 10] = np.nan                                  # a NaN series in the last chunk
    out = np.full_like(x, 7.0)
    c, coef = np.empty(S), np.empty((S, 5))
    lib().sts_ar_fit_remove_host(P(x), P(out), S, T, T, 5, 0, P(c), P(coef), None)   # status: either way
    small = np.ascontiguousarray(x[:37])
    o2, c2, k2, _ = call_ar_fit_remove_host(small)
    assert bits(o2, out[:37]) and bits(c2, c[:37]) and bits(k2, coef[:37])
    # a call that fails validation after a large one leaves the next call intact too
    assert lib().sts_ar_fit_remove_host(P(x), P(x), S, T, T, 5, 0, P(c), P(coef), None) != 0   # alias
    o3, c3, k3, _ = call_ar_fit_remove_host(small)
    assert bits(o3, o2) and bits(c3, c2) and bits(k3, k2)
