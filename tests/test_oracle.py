"""The oracle (CPU restatement) pinned against the reference's own vectors.

Runs on CPU.  Pins, in order of strength:
  * the reference's toeplitz_hash compiled from its source (oracle/_ref) on
    random tuples — skipped where the reference is not mounted;
  * the Intel 82599 verification suite held by dpdk/test/test/test_thash.c;
  * SURVEY.md §8(a)'s known answers from the reference toeplitz_dispatch;
  * the committed synth fixtures (hashes produced by the reference engine).
"""
import json

import numpy as np
import pytest

from frames import ipv4_frame


def test_key_matches_reference(oracle_mod):
    R = oracle_mod.ref()
    if R is None:
        pytest.skip("oracle/_ref not built (reference not mounted)")
    key = bytes(R.ref_default_rsskey()[i] for i in range(40))
    assert key == oracle_mod.MLX_KEY


def test_engine_vs_reference_random(oracle_mod):
    R = oracle_mod.ref()
    if R is None:
        pytest.skip("oracle/_ref not built (reference not mounted)")
    rng = np.random.default_rng(7)
    keys = [oracle_mod.MLX_KEY, bytes(rng.integers(0, 256, 40, dtype=np.uint8))]
    for key in keys:
        for dl in (1, 4, 8, 12, 36):
            for kl in (4, 13, 40):
                for _ in range(50):
                    d = bytes(rng.integers(0, 256, dl, dtype=np.uint8))
                    assert (oracle_mod.lib().oracle_toeplitz_hash(kl, key, dl, d)
                            == R.ref_toeplitz_hash(kl, key, dl, d))


def test_82599_vectors(oracle_mod, golden_dir):
    g = json.loads((golden_dir / "thash_82599.json").read_text())
    key = bytes.fromhex(g["key"])
    for v in g["v4"] + g["v6"]:
        assert oracle_mod.toeplitz_hash(bytes.fromhex(v["l3"]), key) == v["hash_l3"]
        assert oracle_mod.toeplitz_hash(bytes.fromhex(v["l3l4"]), key) == v["hash_l3l4"]


def test_survey_kat(oracle_mod, golden_dir):
    g = json.loads((golden_dir / "survey_kat.json").read_text())
    cfgs = {k: oracle_mod.cfg(*v) for k, v in g["configs"].items()}
    for case in g["cases"]:
        f = bytes.fromhex(case["frame"])
        for cname, want in case["expect"].items():
            if cname == "hash":
                q, h = oracle_mod.toeplitz_dispatch(f, case["len"], cfgs["np8"])
                assert h == want, case["name"]
            else:
                q, _ = oracle_mod.toeplitz_dispatch(f, case["len"], cfgs[cname])
                assert q == want, (case["name"], cname)


def test_table_engine_equals_bit_serial(oracle_mod):
    for profile in range(7):
        win, lens = oracle_mod.synth(profile, 2000, stride=80)
        c = oracle_mod.cfg(8, 8, 1, 0)
        q0, h0 = oracle_mod.dispatch_windows(win, 80, lens, c, fast=False)
        q1, h1 = oracle_mod.dispatch_windows(win, 80, lens, c, fast=True)
        assert np.array_equal(q0, q1) and np.array_equal(h0, h1)


@pytest.mark.parametrize("name", ["udp4_1flow", "udp4", "imix", "vlan6_tcp", "jumbo_tcp4",
                                  "tcp4", "fuzz"])
def test_synth_fixtures(oracle_mod, golden_dir, name):
    d = np.load(golden_dir / f"synth_{name}.npz")
    seed, profile, nflows, stride = (int(x) for x in d["meta"])
    n = d["len"].size
    win, lens = oracle_mod.synth(profile, n, 0, seed, nflows, stride)
    # generator is stable (same header file on host and device)
    assert np.array_equal(win.reshape(n, stride), d["win"])
    assert np.array_equal(lens, d["len"])
    for cname, (npr, nq, soft, only) in {"np8": (8, 8, 1, 0), "ini": (3, 3, 1, 1)}.items():
        c = oracle_mod.cfg(npr, nq, soft, only)
        q, h = oracle_mod.dispatch_windows(win, stride, lens, c)
        assert np.array_equal(q, d[f"q_{cname}"])
        assert np.array_equal(h, d[f"hash_{cname}"])
        qi, qs = oracle_mod.process_burst(q, nq)
        assert np.array_equal(qi, d[f"qidx_{cname}"])
        assert np.array_equal(qs, d[f"qstart_{cname}"])


def test_process_burst_semantics(oracle_mod):
    # drop = ret < 0 || ret >= nb_queues (ff_dpdk_if.c:1080-1083); FIFO per queue
    q = np.array([2, 0, 5, 2, -1, 1, 2, 3, 0, -2], np.int16)
    qi, qs = oracle_mod.process_burst(q, 3)
    buckets = [list(qi[qs[b]:qs[b + 1]]) for b in range(4)]
    assert buckets == [[1, 8], [5], [0, 3, 6], [2, 4, 7, 9]]
    assert qs[-1] == len(q)


def test_length_and_ihl_edges(oracle_mod):
    c = oracle_mod.cfg(8, 8, 1, 0)
    base = ("10.0.0.1", 12345, "10.0.0.2", 80)
    # ip_payload_len = len - ihl4 (NOT minus 14): len 39 with IHL=5 → 19 < 20 → 2
    assert oracle_mod.toeplitz_dispatch(ipv4_frame(*base), 39, c)[0] == 2
    assert oracle_mod.toeplitz_dispatch(ipv4_frame(*base), 40, c)[0] == 6
    # IHL 1..4 accepted (version nibble unchecked)
    for ihl in range(0, 5):
        q, h = oracle_mod.toeplitz_dispatch(ipv4_frame(*base, ihl=ihl), 64, c)
        assert h != 0 and 0 <= q < 8
    # IHL 12 with len 64: ip_len 50 < 48? no; len-ihl4 = 16 < 20 → 2
    assert oracle_mod.toeplitz_dispatch(ipv4_frame(*base, ihl=12), 64, c)[0] == 2
    # IHL 12 with len 80: hashed, ports at 62..65
    q, h = oracle_mod.toeplitz_dispatch(ipv4_frame(*base, ihl=12, length=80), 80, c)
    assert h == 0x0AD63BA6 and q == 6


def test_ff_rss_check_network_order(oracle_mod):
    # ff_rss_check hashes raw network-order fields: with the 82599 key and the
    # 82599 tuple it reproduces the datasheet L3+L4 hash's RETA bits.
    import socket
    import struct

    key = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c"
                        "6a42b73bbeac01fa")
    c = oracle_mod.cfg(4, 4, 1, 0, key=key)
    s = struct.unpack("<I", socket.inet_aton("66.9.149.187"))[0]
    d = struct.unpack("<I", socket.inet_aton("161.142.100.80"))[0]
    sp = struct.unpack("<H", struct.pack(">H", 2794))[0]
    dp = struct.unpack("<H", struct.pack(">H", 1766))[0]
    h = 0x51CCC178
    want_q = (h & 127) % 4
    for qid in range(4):
        got = oracle_mod.lib().oracle_ff_rss_check(c, 4, 128, qid, s, d, sp, dp)
        assert got == (1 if qid == want_q else 0)
