"""The F-Stack config knobs the soft-RSS path reads, parsed from an fs/lib INI.

Mirrors the subset of fs/lib/ff_config.c that feeds toeplitz_dispatch /
process_packets:

* ``[dpdk] lcore_mask``   hex mask; nb_procs = number of set bits
  (ff_config.c:88-136, ``cfg->dpdk.nb_procs = count`` at :133)
* ``[dpdk] soft_dispatch`` (ff_config.c:440-441)
* ``[system] dispatch_only_core`` (ff_config.c:450-451, default 0 at :625)
* ``[portN] lcore_list``  list/range syntax; a port's nb_queues is its lcore
  count, defaulting to all nb_procs lcores (ff_config.c:296-310, :359-367;
  ff_dpdk_if.c:420 ``nb_queue_list[port_id] = nb_lcores``)

Errors follow the reference's init-time behaviour: a bad value is rejected
(ValueError), since ff_load_config fails and rte_exit follows.
"""
from __future__ import annotations

import configparser
from dataclasses import dataclass

RTE_MAX_LCORE = 128


@dataclass
class FfDispatchConfig:
    nb_procs: int
    soft_dispatch: int
    dispatch_only_core: int
    nb_queues: dict  # port id -> nb_queues
    lcore_list: dict  # port id -> sorted lcore ids


def parse_lcore_mask(mask: str) -> list[int]:
    """Lcore ids set in a hex mask, lowest first (ff_config.c:88-131)."""
    m = mask.strip()
    if m.lower().startswith("0x"):
        m = m[2:]
    if not m or any(c not in "0123456789abcdefABCDEF" for c in m):
        raise ValueError(f"invalid lcore_mask {mask!r}")
    val = int(m, 16)
    ids = [i for i in range(RTE_MAX_LCORE) if (val >> i) & 1]
    if val >> RTE_MAX_LCORE:
        raise ValueError(f"lcore_mask {mask!r} exceeds RTE_MAX_LCORE")
    return ids


def parse_list(value: str, max_ele: int = RTE_MAX_LCORE) -> list[int]:
    """'0-3,5,7-8' → [0,1,2,3,5,7,8] (ff_config.c:246-306 __parse_config_list)."""
    out: list[int] = []
    for part in value.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = (int(x) for x in part.split("-", 1))
            if lo > hi:
                raise ValueError(f"bad range {part!r}")
            out.extend(range(lo, hi + 1))
        else:
            out.append(int(part))
        if len(out) > max_ele:
            raise ValueError(f"too many elements in list {value!r}")
    return sorted(out)


def load_ff_config(path: str) -> FfDispatchConfig:
    cp = configparser.ConfigParser(inline_comment_prefixes=(";", "#"), strict=False)
    with open(path) as f:
        cp.read_file(f)
    if not cp.has_option("dpdk", "lcore_mask"):
        raise ValueError("[dpdk] lcore_mask is required")
    lcores = parse_lcore_mask(cp.get("dpdk", "lcore_mask"))
    nb_procs = len(lcores)
    if nb_procs == 0:
        raise ValueError("lcore_mask selects no lcore")
    soft = int(cp.get("dpdk", "soft_dispatch", fallback="0"))
    only = int(cp.get("system", "dispatch_only_core", fallback="0"))
    ports = parse_list(cp.get("dpdk", "port_list", fallback="0"))
    nbq, lists = {}, {}
    for p in ports:
        sec = f"port{p}"
        if cp.has_option(sec, "lcore_list"):
            lst = parse_list(cp.get(sec, "lcore_list"))
        else:
            lst = list(lcores)
        nbq[p] = len(lst)
        lists[p] = lst
    return FfDispatchConfig(nb_procs, soft, only, nbq, lists)
