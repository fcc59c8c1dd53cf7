"""GPU parity for SURVEY §8(f) ranks 4 and 1: the protocol_filter / KNI class
fused into the parse kernel, and yrss_route_burst's process_packets hand-off
(FIFO ring enqueue, drops, ARP clone-to-all, KNI), both against the oracle."""
import struct

import numpy as np
import pytest

from frames import ipv4_frame
from test_gpu_parity import _fake_mbufs, to_np
from test_kni_oracle import ipip_frame

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

KNI_CFGS = [
    (True, "accept", "0-32767", "1000-40000,53,123"),
    (True, "reject", "80,443,8000-8080", None),
    (False, "reject", "0-65535", "0-65535"),
    (True, "accept", None, None),
]


@pytest.mark.parametrize("kcfg", KNI_CFGS)
@pytest.mark.parametrize("stride", [64, 80, 128])
def test_filter_parity_fuzz(oracle_mod, kcfg, stride):
    enable, method, tcp, udp = kcfg
    n = 60001
    with SoftRss(8, 8, 1, 0, device=0, max_burst=0) as eng:
        eng.set_kni(enable, method, tcp, udp)
        for profile in (abi.SYN_FUZZ, abi.SYN_IMIX):
            win, lens = eng.synth(profile, n, 99, stride=stride)
            res = eng.dispatch_dev(win, lens, stride, n, want_filter=True)
            torch.cuda.synchronize()
            w_h = win[: n * stride].cpu().numpy()
            l_h = to_np(lens[:n], np.uint16)
            want = oracle_mod.filter_windows(w_h, stride, l_h, enable,
                                             oracle_mod.kni_bitmap(tcp), oracle_mod.kni_bitmap(udp))
            got = res.filter[:n].cpu().numpy()
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
            # the fused filter leaves the dispatch outputs untouched
            q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, oracle_mod.cfg(8, 8, 1, 0))
            assert np.array_equal(to_np(res.q[:n], np.int16), q_ref)
            assert np.array_equal(to_np(res.hash[:n], np.uint32), h_ref)
            # and the per-queue lists, with no device guard fired
            assert eng.fault_info()[0] == abi.FAULT_NONE
            qi_ref, qs_ref = oracle_mod.process_burst(q_ref, 8)
            assert np.array_equal(to_np(res.qstart, np.uint32), qs_ref)
            assert np.array_equal(to_np(res.qidx[:n], np.uint32), qi_ref)
            if enable and (tcp or udp) and profile == abi.SYN_FUZZ:
                assert (want == abi.FILTER_KNI).sum() > 0 and (want == abi.FILTER_ARP).sum() > 0


def test_filter_ipip_and_edges(oracle_mod):
    frames = []
    for outer in (5, 6, 10, 13, 15):
        for inner in (0, 1, 5, 7):
            for proto in (6, 17, 4, 1):
                for L in (60, 80, 100, 1500):
                    frames.append((ipip_frame(inner, proto, 80, outer_ihl=outer,
                                              length=max(L, 100)), L))
    frames.append((ipv4_frame("1.1.1.1", 1, "2.2.2.2", 80, ihl=12, length=100), 100))
    frames.append((ipv4_frame("1.1.1.1", 1, "2.2.2.2", 80, ihl=12, length=100, proto=17), 100))
    tcp, udp = oracle_mod.kni_bitmap("80"), oracle_mod.kni_bitmap("80,53")
    for stride in (64, 80, 128):
        n = len(frames)
        w = np.zeros((n, stride), np.uint8)
        for i, (f, L) in enumerate(frames):
            b = np.frombuffer(f[:stride], np.uint8)
            w[i, : b.size] = b
        l_h = np.array([L for _, L in frames], np.uint16)
        want = oracle_mod.filter_windows(w.reshape(-1), stride, l_h, True, tcp, udp)
        assert (want == abi.FILTER_LOOP).any() and (want == abi.FILTER_KNI).any()
        with SoftRss(8, device=0, max_burst=0) as eng:
            eng.set_kni(True, "accept", "80", "80,53")
            res = eng.dispatch_dev(torch.from_numpy(w.reshape(-1)).cuda(),
                                   torch.from_numpy(l_h.view(np.int16)).cuda(), stride, n,
                                   want_filter=True)
            torch.cuda.synchronize()
            assert eng.status() == 0
            assert np.array_equal(res.filter[:n].cpu().numpy(), want)


def test_set_kni_rejects_bad_method():
    with SoftRss(3, device=0, max_burst=0) as eng:
        with pytest.raises(abi.YrssError):
            eng.set_kni(True, "drop", "80", None)
        with pytest.raises(abi.YrssError):
            eng.set_kni(True, None, "80", None)
        eng.set_kni(False, None, None, None)


class Rings:
    """Callback side of yrss_route_burst: bounded FIFO rings + clone pool."""

    def __init__(self, addr_to_idx, capacity, clone_ok):
        self.addr_to_idx = addr_to_idx
        self.free = list(capacity)
        self.rings = {j: [] for j in range(len(capacity))}
        self.clone_ok = clone_ok
        self.clones = {}
        self.next_clone = 0x7F0000000000
        self.released = []

    def obj(self, a):
        return self.clones[a] if a in self.clones else ("pkt", self.addr_to_idx[a])

    def enqueue(self, queue, objs):
        k = min(self.free[queue], len(objs))
        self.rings[queue] += [self.obj(a) for a in objs[:k]]
        self.free[queue] -= k
        return k

    def clone(self, m, queue):
        i = self.addr_to_idx[m]
        if not self.clone_ok(i, queue):
            return 0
        self.next_clone += 64
        self.clones[self.next_clone] = ("clone", i, queue)
        return self.next_clone

    def release(self, m):
        self.released.append(self.obj(m))


@pytest.mark.parametrize("queue_id", [0, 1])
@pytest.mark.parametrize("kni", [(False, "reject"), (True, "accept"), (True, "reject")])
@pytest.mark.parametrize("cap", [10**6, 300])
@pytest.mark.parametrize("n", [3000, 6000])   # one-launch small path / multi-kernel path
def test_route_burst_vs_process_packets(oracle_mod, queue_id, kni, cap, n):
    nq = 4
    win, lens = oracle_mod.synth(abi.SYN_FUZZ, n, 5, stride=80)
    frames = []
    for i in range(n):
        L = min(int(lens[i]), 2048)
        f = win[i * 80:(i + 1) * 80].tobytes()
        frames.append((f + bytes(max(0, L - 80)))[:L])
    pool, ptrs, stride = _fake_mbufs(frames)
    addr_to_idx = {int(a): i for i, a in enumerate(ptrs)}
    clone_ok = lambda i, j: (i * 7 + j) % 5 != 0          # noqa: E731 — some clones fail
    capacity = [cap] * nq
    enable, method = kni
    tcp_ports, udp_ports = "0-30000", "20000-65535"
    # oracle: per-packet q and filter class on the full frames, then the model
    c = oracle_mod.cfg(6, nq, 1, 0)
    tcp_bm, udp_bm = oracle_mod.kni_bitmap(tcp_ports), oracle_mod.kni_bitmap(udp_ports)
    q_ref = [oracle_mod.toeplitz_dispatch(f, len(f), c)[0] for f in frames]
    f_ref = [oracle_mod.protocol_filter(f, len(f), enable, tcp_bm, udp_bm, avail=80)
             for f in frames]
    rings_ref, local_ref, kni_ref, freed_ref = oracle_mod.process_packets_route(
        q_ref, f_ref, nq, queue_id, enable, method == "accept", True, capacity, clone_ok)
    with SoftRss(6, nq, 1, 0, device=0) as eng:
        eng.set_kni(enable, method, tcp_ports, udp_ports)
        cb = Rings(addr_to_idx, capacity, clone_ok)
        local, kni_list, res = eng.route_burst(ptrs, queue_id, cb.enqueue, cb.clone, cb.release)
    assert cb.rings == rings_ref
    assert [cb.obj(a) for a in local] == local_ref
    assert [cb.obj(a) for a in kni_list] == kni_ref
    assert sorted(cb.released) == sorted(freed_ref)
    assert res.n_freed == len(freed_ref)
    assert res.n_unresolved == sum(1 for o in local_ref if f_ref[o[1]] in (-2, -3))
    assert [res.n_ring[j] for j in range(nq)] == [len(rings_ref[j]) for j in range(nq)]


def test_from_ff_config_kni(oracle_mod, tmp_path):
    """[kni] keys read from an fs/lib INI (ff_config.c:442-449) configure the
    fused filter exactly as init_kni would (ff_dpdk_if.c:598-606)."""
    ini = tmp_path / "kni.ini"
    ini.write_text("[dpdk]\nlcore_mask=f\nsoft_dispatch=1\nport_list=0\n[system]\n"
                   "dispatch_only_core=1\n[kni]\nenable=1\nmethod=accept\n"
                   "tcp_port=80,443,8000-8080\nudp_port=53 ; dns\n[port0]\naddr=10.0.0.2\n"
                   "netmask=255.255.255.0\nbroadcast=10.0.0.255\ngateway=10.0.0.1\n"
                   "lcore_list=0-3\n")
    n, stride = 30001, 80
    with SoftRss.from_ff_config(str(ini), device=0, max_burst=0) as eng:
        assert (eng.cfg.nb_procs, eng.nb_queues) == (4, 4)
        win, lens = eng.synth(abi.SYN_FUZZ, n, 5, stride=stride)
        res = eng.dispatch_dev(win, lens, stride, n, want_filter=True)
        torch.cuda.synchronize()
        w_h = win[: n * stride].cpu().numpy()
        l_h = to_np(lens[:n], np.uint16)
        want = oracle_mod.filter_windows(w_h, stride, l_h, True,
                                         oracle_mod.kni_bitmap("80,443,8000-8080"),
                                         oracle_mod.kni_bitmap("53"))
        assert np.array_equal(res.filter[:n].cpu().numpy(), want)
        q_ref, _ = oracle_mod.dispatch_windows(w_h, stride, l_h, oracle_mod.cfg(4, 4, 1, 1))
        assert np.array_equal(to_np(res.q[:n], np.int16), q_ref)
        assert eng.status() == 0
        qi_ref, qs_ref = oracle_mod.process_burst(q_ref, 4)
        assert np.array_equal(to_np(res.qstart, np.uint32), qs_ref)
        assert np.array_equal(to_np(res.qidx[:n], np.uint32), qi_ref)
