"""The F-Stack config knobs the soft-RSS path reads, parsed from an fs/lib INI
exactly as fs/lib reads them.

Two layers, each restating the reference:

* :func:`ini_parse` — the INI reader F-Stack vendors (inih, fs/lib/ff_ini_parser.c
  :73-172 with the options of ff_ini_parser.h:54-90): ``fgets`` lines of at most
  199 bytes (INI_MAX_LINE 200), a UTF-8 BOM skipped, ``;``/``#`` comment lines,
  ``;`` inline comments only after whitespace, ``name=value`` or ``name:value``,
  continuation lines (leading whitespace) re-sent under the previous name,
  section names cut to 49 bytes, and parsing stops at the first error, whose
  line number is returned (0 = success).  Names and sections are
  case-sensitive.  ``tests/test_ffconfig.py`` checks it event for event against
  the reference parser itself (``oracle/_ref/libref_ini.so``, compiled from
  ff_ini_parser.c where it lies).
* :func:`load_ff_config` — the part of ``ini_parse_handler``
  (fs/lib/ff_config.c:410-469) that feeds toeplitz_dispatch / process_packets
  and the KNI filter, plus ``ff_check_config``'s checks on it (:538-604):

  - ``[dpdk] lcore_mask``: parse_lcore_mask (:73-136), nb_procs = set bits (:133)
  - ``[dpdk] port_list``, ``[portN] lcore_list``: __parse_config_list (:246-308)
    over rte_strsplit (dpdk/lib/librte_eal/common/eal_common_string_fns.c:14-40);
    a port's nb_queues is its lcore count, all nb_procs lcores unless listed
    (:355-367, ff_dpdk_if.c:420)
  - ``[dpdk] soft_dispatch`` (:440-441), ``[system] dispatch_only_core`` (:450-451)
  - ``[kni] enable / method / tcp_port / udp_port`` (:442-449), consumed by
    init_kni (ff_dpdk_if.c:598-606, :921-923)

Errors follow the reference's init-time behaviour: where ff_load_config fails
(and rte_exit follows) this raises ValueError naming the line or the check.
"""
from __future__ import annotations

from dataclasses import dataclass, field

RTE_MAX_LCORE = 128       # parse_lcore_mask's bit limit (build config)
DPDK_MAX_LCORE = 128      # fs/lib/ff_config.h:40
RTE_MAX_ETHPORTS = 32     # dpdk/config/rte_config.h:46
INI_MAX_LINE = 200        # ff_ini_parser.h:88-90
MAX_SECTION = 50          # ff_ini_parser.c:24-25
MAX_NAME = 50
_SPACE = b" \t\n\v\f\r"   # isspace() in the C locale
_BLANK = b" \t"           # isblank()


# ---- inih (fs/lib/ff_ini_parser.c) ----------------------------------------------
def _fgets_lines(data: bytes):
    """fgets(line, INI_MAX_LINE, f): up to 199 bytes, through the newline."""
    pos = 0
    while pos < len(data):
        nl = data.find(b"\n", pos)
        end = len(data) if nl < 0 else nl + 1
        end = min(end, pos + INI_MAX_LINE - 1)
        yield data[pos:end]
        pos = end


def _find_chars_or_comment(s: bytes, chars: bytes | None) -> int:
    """Index of the first of `chars`, or of a ';' that follows whitespace (:47-62)."""
    was_space = False
    for i, c in enumerate(s):
        if (chars is not None and c in chars) or (was_space and c == ord(";")):
            return i
        was_space = c in _SPACE
    return len(s)


def ini_parse(data: bytes, handler) -> int:
    """ini_parse_stream (:73-172).  handler(section, name, value) -> bool, all
    str (bytes decoded latin-1).  Returns 0, or the first error's line."""
    section = b""
    prev_name = b""
    lineno = 0
    for raw in _fgets_lines(data):
        lineno += 1
        line = raw.split(b"\0", 1)[0]            # C strings end at the first NUL
        start = 3 if lineno == 1 and line[:3] == b"\xef\xbb\xbf" else 0
        body = line[start:].rstrip(_SPACE)
        stripped = body.lstrip(_SPACE)
        indented = start > 0 or len(stripped) != len(body)
        err = False
        if stripped[:1] in (b";", b"#"):
            pass
        elif prev_name and stripped and indented:
            # continuation of the previous name's value (INI_ALLOW_MULTILINE)
            err = not handler(section.decode("latin-1"), prev_name.decode("latin-1"),
                              stripped.decode("latin-1"))
        elif stripped[:1] == b"[":
            end = _find_chars_or_comment(stripped[1:], b"]") + 1
            if end < len(stripped) and stripped[end:end + 1] == b"]":
                section = stripped[1:end][:MAX_SECTION - 1]
                prev_name = b""
            else:
                err = True
        elif stripped:
            end = _find_chars_or_comment(stripped, b"=:")
            if stripped[end:end + 1] in (b"=", b":"):
                name = stripped[:end].rstrip(_SPACE)
                value = stripped[end + 1:]
                value = value[:_find_chars_or_comment(value, None)]
                value = value.lstrip(_SPACE).rstrip(_SPACE)
                prev_name = name[:MAX_NAME - 1]
                err = not handler(section.decode("latin-1"), name.decode("latin-1"),
                                  value.decode("latin-1"))
            else:
                err = True
        if err:                                  # INI_STOP_ON_FIRST_ERROR
            return lineno
    return 0


def ini_events(data: bytes):
    """(events, error): every (section, name, value) the reader hands out."""
    ev = []
    err = ini_parse(data, lambda s, n, v: ev.append((s, n, v)) or True)
    return ev, err


# ---- C conversions the handler uses --------------------------------------------
def c_atoi(s: str) -> int:
    """atoi(): leading whitespace, sign, digits; anything else stops it."""
    i, n = 0, len(s)
    while i < n and s[i] in " \t\n\v\f\r":
        i += 1
    sign = 1
    if i < n and s[i] in "+-":
        sign = -1 if s[i] == "-" else 1
        i += 1
    v = 0
    while i < n and s[i].isdigit() and s[i].isascii():
        v = v * 10 + ord(s[i]) - 48
        i += 1
    v *= sign
    return ((v + 2**31) % 2**32) - 2**31


def _c_strtol_full(s: str) -> int | None:
    """strtol(s, &end, 10) with *end == '\\0' required; None when it is not."""
    i, n = 0, len(s)
    while i < n and s[i] in " \t\n\v\f\r":
        i += 1
    j = i
    if j < n and s[j] in "+-":
        j += 1
    k = j
    while k < n and "0" <= s[k] <= "9":
        k += 1
    if k == j:                 # no digits: end = s, so only the empty string passes
        return 0 if n == 0 else None
    if k != n:
        return None
    return int(s[i:k])


# ---- ff_config.c handlers ------------------------------------------------------
def parse_lcore_mask(mask: str, proc_id: int = 0) -> list[int]:
    """parse_lcore_mask (ff_config.c:73-136): lcore ids set in a hex mask,
    lowest first.  ValueError where the reference returns 0."""
    m = mask.lstrip(" \t")
    if m[:2] in ("0x", "0X"):
        m = m[2:]
    m = m.rstrip(" \t")
    if not m:
        raise ValueError(f"invalid lcore_mask {mask!r}")
    ids = []
    idx = 0
    i = len(m) - 1
    while i >= 0 and idx < RTE_MAX_LCORE:
        c = m[i]
        if c not in "0123456789abcdefABCDEF":
            raise ValueError(f"invalid lcore_mask {mask!r}")
        val = int(c, 16)
        for j in range(4):
            if idx >= RTE_MAX_LCORE:
                break
            if (val >> j) & 1:
                ids.append(idx)
            idx += 1
        i -= 1
    if any(c != "0" for c in m[: i + 1]):
        raise ValueError(f"lcore_mask {mask!r} exceeds RTE_MAX_LCORE")
    if proc_id >= len(ids):
        raise ValueError(f"proc_id {proc_id} not in lcore_mask {mask!r}")
    return ids


def _strsplit(s: str, maxtokens: int = 128) -> list[str]:
    """rte_strsplit(.., ','): a trailing ',' adds no token, an inner empty
    field does; once maxtokens are open the last one keeps the rest."""
    chars = list(s)
    starts, tokstart = [], True
    for i, c in enumerate(chars):
        if len(starts) >= maxtokens:
            break
        if tokstart:
            tokstart = False
            starts.append(i)
        if c == ",":
            chars[i] = "\0"
            tokstart = True
    t = "".join(chars)
    return [t[i:].split("\0", 1)[0] for i in starts]


def parse_list(value: str, max_ele: int = DPDK_MAX_LCORE) -> list[int]:
    """__parse_config_list (ff_config.c:246-308): '0-3,5' -> [0,1,2,3,5], as
    uint16 values, sorted.  The reference's bound check admits max_ele + 1
    elements; an empty list leaves the reference's size at its maximum
    (undefined contents), which is rejected here."""
    out: list[int] = []
    for tok in _strsplit(value[:4096]):
        if "-" not in tok:
            v = _c_strtol_full(tok.strip(" "))
            if v is None:
                raise ValueError(f"{tok!r} is not a integer")
            if len(out) > max_ele:
                raise ValueError(f"too many elements in list {value!r}")
            out.append(v & 0xFFFF)
        else:
            lo_s, hi_s = tok.split("-", 1)
            lo, hi = _c_strtol_full(lo_s.strip(" ")), _c_strtol_full(hi_s.strip(" "))
            if lo is None or hi is None:
                raise ValueError(f"{tok!r} is not a integer range")
            for j in range(lo, hi + 1):
                if len(out) > max_ele:
                    raise ValueError(f"too many elements in list {value!r}")
                out.append(j & 0xFFFF)
    if not out:
        raise ValueError(f"list {value!r} is empty")
    return sorted(out)


@dataclass
class FfPortConfig:
    port_id: int
    lcore_list: list
    addr: str | None = None
    netmask: str | None = None
    broadcast: str | None = None
    gateway: str | None = None
    hardware_rss: int = 0


@dataclass
class FfDispatchConfig:
    nb_procs: int
    soft_dispatch: int
    dispatch_only_core: int
    nb_queues: dict          # port id -> nb_queues (the port's lcore count)
    lcore_list: dict         # port id -> sorted lcore ids
    proc_lcore: list = field(default_factory=list)
    kni_enable: int = 0
    kni_method: str | None = None
    kni_tcp_port: str | None = None
    kni_udp_port: str | None = None

    @property
    def kni_accept(self) -> bool:
        """init_kni: strcasecmp(method, "accept") == 0 (ff_dpdk_if.c:601-603)."""
        return (self.kni_method or "").lower() == "accept"


def load_ff_config(path: str, proc_id: int = 0, check: bool = True) -> FfDispatchConfig:
    """Parse an fs/lib INI as ff_load_config does (ff_config.c:629-650) and
    return the soft-RSS knobs.  ``check`` applies ff_check_config (:538-604)."""
    with open(path, "rb") as f:
        data = f.read()
    st = {"lcores": None, "soft": 0, "only": 0, "ports": None, "max_port": -1,
          "pcfg": None, "kni_enable": 0, "kni_method": None, "kni_tcp": None,
          "kni_udp": None}

    def port_handler(section, name, value):
        # port_cfg_handler (ff_config.c:341-405)
        if not st["ports"]:
            return False                       # "must config dpdk.port_list first"
        if st["pcfg"] is None:
            lc = st["lcores"] or []
            st["pcfg"] = {p: FfPortConfig(p, list(lc)) for p in st["ports"]}
        num = section[4:].lstrip(" \t\n\v\f\r")
        k = 1 if num[:1] in ("+", "-") else 0
        d0 = k
        while k < len(num) and "0" <= num[k] <= "9":
            k += 1
        if k == d0:
            return False                       # sscanf("port%d") != 1
        portid = int(num[:k])
        if portid > st["max_port"]:
            return True                        # ignored: beyond max_portid
        # a port absent from port_list has a zeroed entry (calloc, :352-368)
        pc = st["pcfg"].setdefault(portid, FfPortConfig(portid, []))
        if name in ("addr", "netmask", "broadcast", "gateway"):
            setattr(pc, name, value)
        elif name == "lcore_list":
            try:
                pc.lcore_list = parse_list(value, DPDK_MAX_LCORE)
            except ValueError:
                return False
        elif name == "hardware_rss":
            pc.hardware_rss = c_atoi(value)
        return True

    def handler(section, name, value):
        # ini_parse_handler (ff_config.c:410-469), the keys this path reads
        if section == "dpdk" and name == "lcore_mask":
            try:
                st["lcores"] = parse_lcore_mask(value, proc_id)
            except ValueError:
                return False
        elif section == "dpdk" and name == "port_list":
            try:
                ports = parse_list(value, RTE_MAX_ETHPORTS)
            except ValueError:
                return False
            st["ports"], st["max_port"] = ports, ports[-1]
        elif section == "dpdk" and name == "soft_dispatch":
            st["soft"] = c_atoi(value)
        elif section == "kni" and name == "enable":
            st["kni_enable"] = c_atoi(value)
        elif section == "kni" and name == "method":
            st["kni_method"] = value
        elif section == "kni" and name == "tcp_port":
            st["kni_tcp"] = value
        elif section == "kni" and name == "udp_port":
            st["kni_udp"] = value
        elif section == "system" and name == "dispatch_only_core":
            st["only"] = c_atoi(value)
        elif section.startswith("port"):
            return port_handler(section, name, value)
        return True

    err = ini_parse(data, handler)
    if err:
        raise ValueError(f"{path}: parse error at line {err}")
    if not st["lcores"]:
        raise ValueError(f"{path}: [dpdk] lcore_mask is required")
    ports = st["ports"] or []
    pcfg = st["pcfg"] or {}
    if check:
        # ff_check_config (ff_config.c:538-604)
        if st["kni_enable"] and not st["kni_method"]:
            raise ValueError("conf dpdk.method is necessary")
        if st["kni_method"] and st["kni_method"].lower() not in ("accept", "reject"):
            raise ValueError(f"conf kni.method[accept|reject] is error({st['kni_method']})")
        if ports and not pcfg:
            raise ValueError("no [portN] section")
        for p in ports:
            pc = pcfg.get(p)
            for f in ("addr", "netmask", "broadcast", "gateway"):
                if pc is None or getattr(pc, f) is None:
                    raise ValueError(f"port{p} if config error: no {f}")
            for lc in pc.lcore_list:
                if lc not in st["lcores"]:
                    raise ValueError(f"lcore {lc} is not enabled.")
            if st["kni_enable"] and st["lcores"][proc_id] not in pc.lcore_list:
                raise ValueError(f"primary lcore {st['lcores'][proc_id]} should stay in "
                                 f"port {p}'s lcore_list.")
    lists = {p: (pcfg[p].lcore_list if p in pcfg else list(st["lcores"])) for p in ports}
    return FfDispatchConfig(
        nb_procs=len(st["lcores"]), soft_dispatch=st["soft"], dispatch_only_core=st["only"],
        nb_queues={p: len(v) for p, v in lists.items()}, lcore_list=lists,
        proc_lcore=list(st["lcores"]), kni_enable=st["kni_enable"],
        kni_method=st["kni_method"], kni_tcp_port=st["kni_tcp"], kni_udp_port=st["kni_udp"])
