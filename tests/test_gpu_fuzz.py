"""Seeded random configurations through the device path, against the oracle:
nb_procs / nb_queues / soft_dispatch / dispatch_only_core, stream, stride, size
and starting packet drawn at random (40 cases, each small enough for the
oracle).  And two host threads driving their own contexts at once (the GIL is
released inside every ctypes call), each checked against the oracle.
"""
import os
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_parity import _fake_mbufs, run_and_compare  # noqa: E402
from test_gpu_small_burst import _expect, _frames  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


def _cases(count, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < count:
        soft = int(rng.integers(0, 2))
        only = int(rng.integers(0, 2))
        npr = int(rng.choice([1, 2, 3, 4, 7, 8, 17, 33, 64, 255, 4096]))
        if soft and only and npr < 2:
            continue   # rejected by yrss_config_validate (the reference divides by zero)
        nq = int(rng.choice([1, 2, 3, 8, 16, 17, 64, 65, 200, 256]))
        stride = int(rng.choice([64, 80, 96, 128, 2176]))
        profile = int(rng.integers(0, 7))
        n = int(rng.integers(1, 30000))
        first = int(rng.integers(0, 1 << 40))
        out.append((npr, nq, soft, only, stride, profile, n, first))
    return out


# YRSS_FUZZ_CASES / YRSS_FUZZ_SEED widen the sweep for a soak run
@pytest.mark.parametrize("case", _cases(int(os.environ.get("YRSS_FUZZ_CASES", "40")),
                                        int(os.environ.get("YRSS_FUZZ_SEED", "2024"))))
def test_random_configs(dev, oracle_mod, case):
    npr, nq, soft, only, stride, profile, n, first = case
    with SoftRss(npr, nq, soft, only, device=0, max_burst=0) as eng:
        run_and_compare(eng, oracle_mod, (npr, nq, soft, only), profile, n, stride, first=first)


def _large_cases(count, seed):
    # batches of many spans and many scatter ranges (the line scatter's
    # in-scatter prefixes up to 16 buckets, the scan kernel past them), with
    # the prefix form, the XCD mapping and the parse grid drawn as well
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < count:
        npr = int(rng.choice([2, 3, 4, 8, 16, 64, 255]))
        nq = int(rng.choice([1, 2, 3, 4, 7, 15, 16, 17, 64]))
        only = int(rng.integers(0, 2))
        profile = int(rng.choice([1, 2, 4, 5, 6]))
        n = int(rng.integers(1 << 17, 1 << 21))
        first = int(rng.integers(0, 1 << 40))
        tune = (int(rng.integers(0, 2)), int(rng.choice([-1, 0, 1])),
                int(rng.choice([0, 64, 256])))
        out.append((npr, nq, only, profile, n, first, tune))
    return out


@pytest.mark.parametrize("case", _large_cases(int(os.environ.get("YRSS_FUZZ_LARGE_CASES", "6")),
                                              int(os.environ.get("YRSS_FUZZ_SEED", "2024"))))
def test_random_large_batches(dev, oracle_mod, case):
    npr, nq, only, profile, n, first, (scan_kernel, xcd, blocks) = case
    with SoftRss(npr, nq, 1, only, device=0, max_burst=0) as eng:
        eng.set_tuning(scan_kernel=scan_kernel, scatter_xcd=xcd, parse_blocks=blocks)
        run_and_compare(eng, oracle_mod, (npr, nq, 1, only), profile, n, 64, first=first)


def test_two_threads_two_contexts(dev, oracle_mod):
    cfgs = [(3, 3, 1, 1), (8, 6, 1, 0)]
    frames = _frames(oracle_mod, 6000, 77)
    pool, ptrs, _ = _fake_mbufs(frames)
    expect = [_expect(oracle_mod, frames, c) for c in cfgs]
    errors = []

    def run(k):
        try:
            with SoftRss(*cfgs[k], device=0, max_burst=0) as eng:
                eng.register_host_memory(pool.ctypes.data, pool.nbytes)
                rng = np.random.default_rng(k)
                for _ in range(60):
                    n = int(rng.integers(1, 6000))
                    off = int(rng.integers(0, 6000 - n + 1))
                    r = (eng.dispatch_burst_zc(ptrs[off:off + n]) if rng.random() < 0.5
                         else eng.dispatch_burst(ptrs[off:off + n]))
                    q, h, _, _ = expect[k]
                    qi, qs = oracle_mod.process_burst(q[off:off + n], cfgs[k][1])
                    assert np.array_equal(r.q, q[off:off + n])
                    assert np.array_equal(r.hash, h[off:off + n])
                    assert np.array_equal(r.qidx, qi)
                    assert np.array_equal(r.qstart[: qs.size], qs)
                eng.unregister_host_memory(pool.ctypes.data)
        except BaseException as e:   # surfaced in the main thread
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
