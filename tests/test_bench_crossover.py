"""bench.py's end-to-end crossover: the hashed-TCP
share above which a host-resident GPU form beats one reference dispatcher
core.  Host logic only: the CPU's per-packet time is the share-weighted mix
of its UDP and TCP times (the reference hashes TCP only,
fs/lib/ff_dpdk_if.c:1986-2058), the GPU's rate does not depend on the share."""
import bench


def _cpu(udp, tcp):
    return {"by_profile": {"udp4": {"bit_serial_fnptr": {"1": {"mpps": udp}}},
                           "tcp4": {"bit_serial_fnptr": {"1": {"mpps": tcp}}}}}


def test_crossover_share_solves_the_mix():
    x = bench.crossover_tcp_share(_cpu(500.0, 20.0),
                                  [{"api": "yrss_worker_submit_frames", "burst": 32, "mpps": 200.0},
                                   {"api": "yrss_dispatch_burst", "burst": 1024, "mpps": 50.0}])
    assert len(x["rows"]) == 1   # worker forms only
    s = x["rows"][0]["tcp_share"]
    # at that share one core takes exactly the GPU form's time a packet
    assert abs((s / 20.0 + (1 - s) / 500.0) - 1 / 200.0) < 1e-6


def test_crossover_bounds():
    rows = [{"api": "yrss_worker_submit", "burst": 32, "mpps": 900.0},   # faster than all-UDP CPU
            {"api": "yrss_worker_submit", "burst": 1024, "mpps": 10.0}]  # slower than all-TCP CPU
    x = bench.crossover_tcp_share(_cpu(500.0, 20.0), rows)
    assert [r["tcp_share"] for r in x["rows"]] == [0.0, None]
    assert bench.crossover_tcp_share(None, rows) is None
    assert bench.crossover_tcp_share(_cpu(500.0, 20.0), None) is None
