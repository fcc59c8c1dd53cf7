"""pcap capture I/O: the writer produces the byte layout of
F-Stack's dump (fs/lib/ff_dpdk_pcap.c:32-102, restated in oracle.pcap_bytes);
the reader replays any Ethernet capture into dispatch windows.  CPU only — the
GPU replay parity is in test_gpu_parity_pcap below (marked gpu)."""
import struct

import numpy as np
import pytest

from yastack_amd import abi, pcap


def _frames(oracle_mod, n=500, profile=6):
    win, lens = oracle_mod.synth(profile, n, 3, stride=80)
    out = []
    for i in range(n):
        L = min(int(lens[i]), 3000)
        f = win[i * 80:(i + 1) * 80].tobytes()
        out.append((f + bytes(range(256)) * 12)[:L])
    return out


def test_writer_matches_reference_layout(oracle_mod, tmp_path):
    frames = _frames(oracle_mod)
    sec = np.arange(len(frames), dtype=np.uint32) + 1_700_000_000
    usec = (np.arange(len(frames), dtype=np.uint32) * 7919) % 1_000_000
    p = str(tmp_path / "a.pcap")
    pcap.write(p, frames[:200], sec[:200], usec[:200])
    pcap.write(p, frames[200:], sec[200:], usec[200:], append=True)
    assert open(p, "rb").read() == oracle_mod.pcap_bytes(frames, sec, usec)


def test_reader_roundtrip(oracle_mod, tmp_path):
    frames = _frames(oracle_mod)
    p = str(tmp_path / "b.pcap")
    pcap.write(p, frames)
    assert pcap.count(p) == len(frames)
    for stride in (64, 80, 128):
        win, lens, wire = pcap.read(p, stride=stride)
        assert len(lens) == len(frames)
        for i, f in enumerate(frames):
            k = min(len(f), stride)
            assert win[i * stride:i * stride + k].tobytes() == f[:k]
            assert lens[i] == min(len(f), 65535) and wire[i] == len(f)
    win, lens, _ = pcap.read(p, first=123, max_pkts=10)
    assert win[:80].tobytes() == (frames[123] + bytes(80))[:80][:min(80, len(frames[123]))] + \
        bytes(80 - min(80, len(frames[123])))
    assert len(lens) == 10


def test_reader_byte_orders_and_errors(oracle_mod, tmp_path):
    frames = _frames(oracle_mod, 20, profile=5)
    le = oracle_mod.pcap_bytes(frames)
    # big-endian capture of the same frames, nanosecond magic
    be = bytearray(struct.pack(">IHHiIII", 0xA1B23C4D, 2, 4, 0, 0, 65535, 1))
    for f in frames:
        be += struct.pack(">IIII", 1, 2, len(f), len(f)) + f
    for name, blob in (("le.pcap", le), ("be.pcap", bytes(be))):
        p = tmp_path / name
        p.write_bytes(blob)
        win, lens, _ = pcap.read(str(p), stride=80)
        assert [int(x) for x in lens] == [len(f) for f in frames]
    bad = tmp_path / "bad.pcap"
    bad.write_bytes(b"\x00" * 24)
    with pytest.raises(abi.YrssError):
        pcap.read(str(bad))
    with pytest.raises(abi.YrssError):
        pcap.count(str(tmp_path / "missing.pcap"))
    # a truncated last record is an I/O error, not silent garbage
    trunc = tmp_path / "trunc.pcap"
    trunc.write_bytes(le[:-5])
    with pytest.raises(abi.YrssError):
        pcap.read(str(trunc))


@pytest.mark.gpu
def test_gpu_parity_pcap_replay(oracle_mod, tmp_path):
    torch = pytest.importorskip("torch")
    from yastack_amd import SoftRss

    frames = _frames(oracle_mod, 4000) + _frames(oracle_mod, 4000, profile=2)
    p = str(tmp_path / "replay.pcap")
    pcap.write(p, frames)
    win, lens, _ = pcap.read(p, stride=80)
    c = oracle_mod.cfg(3, 3, 1, 1)
    want = [oracle_mod.toeplitz_dispatch(f, len(f), c) for f in frames]
    with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
        res = eng.dispatch_dev(torch.from_numpy(win).cuda(),
                               torch.from_numpy(lens.view(np.int16)).cuda(), 80)
        torch.cuda.synchronize()
        n = len(frames)
        assert res.q[:n].cpu().tolist() == [q for q, _ in want]
        assert res.hash[:n].cpu().numpy().view(np.uint32).tolist() == [h for _, h in want]
