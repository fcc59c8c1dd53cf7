"""Pipelined device batches (yrss_dispatch_dev_pipelined / yrss_dispatch_join):
each batch's per-queue lists are built on the context's lists stream, on CUs
of their own, while the caller's stream goes on to the next batch's parse
kernel.  Every batch must give the oracle's q, hash and per-queue FIFO lists
(fs/lib/ff_dpdk_if.c:1945-2113, :1058-1094) exactly as the plain call does,
with the two workspace sets alternating, batches of different sizes and
bucket counts, plain calls and stream switches in between, and the fault
record empty."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_layout import to_np  # noqa: E402


def _expect(oracle_mod, win, lens, n, stride, cfg):
    npr, nq, soft, only = cfg
    w_h = win[: n * stride].cpu().numpy()
    l_h = to_np(lens[:n], np.uint16)
    q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, oracle_mod.cfg(npr, nq, soft, only))
    qi_ref, qs_ref = oracle_mod.process_burst(q_ref, nq)
    return q_ref, h_ref, qi_ref, qs_ref


def _check(res, n, ref):
    q_ref, h_ref, qi_ref, qs_ref = ref
    assert np.array_equal(to_np(res.q[:n], np.int16), q_ref)
    assert np.array_equal(to_np(res.hash[:n], np.uint32), h_ref)
    assert np.array_equal(to_np(res.qstart, np.uint32), qs_ref)
    assert np.array_equal(to_np(res.qidx[:n], np.uint32), qi_ref)


@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (8, 8, 1, 0), (64, 64, 1, 0), (255, 255, 1, 0)])
def test_pipelined_batches(oracle_mod, cfg):
    sizes = [300001, 1 << 20, 77777, 5000, 1 << 20, 4097]
    stride = 64
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        batches = []
        for i, n in enumerate(sizes):
            prof = (abi.SYN_TCP4, abi.SYN_FUZZ, abi.SYN_IMIX)[i % 3]
            win, lens = eng.synth(prof, n, 1000 * i + 7, stride=stride)
            batches.append((win, lens, n))
        refs = [_expect(oracle_mod, w, l, n, stride, cfg) for w, l, n in batches]
        outs = [eng.dispatch_dev(w, l, stride, n, pipeline=True) for w, l, n in batches]
        eng.join()
        torch.cuda.synchronize()
        assert eng.fault_info()[0] == abi.FAULT_NONE, eng.fault_info()
        for res, (w, l, n), ref in zip(outs, batches, refs):
            _check(res, n, ref)


def test_pipelined_mixed_with_plain_and_streams(oracle_mod):
    """Plain calls, a second stream and pipelined calls interleaved: each
    plain call and each stream switch joins the pending lists first."""
    cfg, stride = (8, 8, 1, 1), 64
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        s2 = torch.cuda.Stream()
        plan = [("p", None), ("p", None), ("plain", None), ("p", s2), ("p", None), ("p", s2),
                ("plain", s2), ("p", None)]
        done = []
        for i, (kind, st) in enumerate(plan):
            n = (1 << 19) + 1000 * i
            win, lens = eng.synth(abi.SYN_IMIX, n, 7777 * i, stride=stride)
            torch.cuda.synchronize()
            res = eng.dispatch_dev(win, lens, stride, n, stream=st, pipeline=(kind == "p"))
            done.append((res, win, lens, n))
        eng.join()
        eng.join(s2)
        torch.cuda.synchronize()
        assert eng.fault_info()[0] == abi.FAULT_NONE, eng.fault_info()
        for res, win, lens, n in done:
            _check(res, n, _expect(oracle_mod, win, lens, n, stride, cfg))


@pytest.mark.parametrize("list_cus", [8, 64])
def test_pipelined_list_cus(oracle_mod, list_cus):
    """The lists stream's CU count is a layout choice only."""
    cfg, stride, n = (64, 64, 1, 1), 64, 1 << 21
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        eng.set_tuning(list_cus=list_cus)
        wins = [eng.synth(abi.SYN_TCP4, n, k * n, stride=stride) for k in range(3)]
        outs = [eng.dispatch_dev(w, l, stride, n, pipeline=True) for w, l in wins]
        eng.join()
        torch.cuda.synchronize()
        assert eng.fault_info()[0] == abi.FAULT_NONE
        for res, (w, l) in zip(outs, wins):
            _check(res, n, _expect(oracle_mod, w, l, n, stride, cfg))
