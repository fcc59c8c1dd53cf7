#!/usr/bin/env python3
"""Build the round-6 measurement-only libraries into ablib/ from a temporary,
edited copy of yastack_amd/csrc/yrss.hip (the tree itself is never edited, and
tests/test_abi.py keeps yrss.hip free of measurement paths).

Each variant is a list of (anchor, replacement) text edits; an anchor that no
longer matches exactly once fails the build of that variant, so a stale edit
cannot silently measure something else.  What the variants measure (DESIGN
section 14):

  noload  span g+1's rank-stream loads replaced by span g's registers (the
          upper bound of what smaller per-packet streams, e.g. bucket codes,
          could save the line scatter)
  noconf  the placement's table reads and stage writes at conflict-free LDS
          addresses (the upper bound of any swizzle)
  pA      the parse kernel with no counting and no ranks
  pB      the parse kernel with no Toeplitz table lookups (a multiply mix)
  pC      hash % d as h & (d - 1) (exact for d a power of two)
  pD      the parse kernel with counts but no ranks
  pf2     two tiles of loads ahead in the parse kernel (three register sets)
  grid1   the line scatter at one workgroup a CU (twice the spans a workgroup)

Lists are wrong by design in noload, noconf, pA and pD; their end-of-range
check is removed so a faulting batch does not time the fault path.

    python tools/build_measure_libs.py noload noconf ...   (default: all)
"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "yastack_amd" / "csrc"

NO_RANGE_CHECK = (
    """        if (misc[3] != want)
            report_fault(P.fault, YRSS_FAULT_COUNT_MISMATCH, YRSS_K_SCATTER, g0, misc[3]);
        else if (misc[1] != want_sum)
            report_fault(P.fault, YRSS_FAULT_STAGE, YRSS_K_SCATTER, g0, misc[1]);""",
    """        (void)want;   // MEASUREMENT: lists wrong by design, no end-of-range check
        (void)want_sum;""")

VARIANTS = {
    "noload": [
        ("""        if (!last)
            load_span(g + 1u, pkn, qkn);
        if (kG != 4u || !misc[8u + s]) {""",
         """        if (!last) {   // MEASUREMENT: no next-span stream loads
            load_span(g + 1u, pkn, qkn, P.fused ? 1u : 3u);
            if (P.fused) {
#pragma unroll
                for (uint32_t k = 0; k < kG; ++k) { pkn[k] = pk[k]; qkn[k] = qk[k]; }
            }
        }
        if (kG != 4u || !misc[8u + s]) {"""),
        NO_RANGE_CHECK,
    ],
    "noconf": [
        ("""                    slot[k - k0][j] = tab[__umul24(b, rs) + cc] + rk;""",
         """                    // MEASUREMENT: conflict-free table read
                    slot[k - k0][j] = tab[(t + (b & 1u) + cc) & 511u] + rk;"""),
        ("""                        stg[min(slot[k - k0][j], cap)] = id + j;""",
         """                        // MEASUREMENT: conflict-free stage write (lanes consecutive)
                        stg[min(((j * kG + k) * kLineBlock + t + (slot[k - k0][j] & 0x80000000u)), cap)] = id + j;"""),
        NO_RANGE_CHECK,
    ],
    "pA": [
        ("""    if (kCount) {
        // per-bucket counts of this chunk: lanes sharing a bucket are found""",
         """    if (false) {   // MEASUREMENT: no counting, no ranks
        // per-bucket counts of this chunk: lanes sharing a bucket are found"""),
        ("""        } else if (leader) {
            atomicAdd(&cnt[bkt], (uint32_t)__popcll(peers));
        }
    }
}""",
         """        } else if (leader) {
            atomicAdd(&cnt[bkt], (uint32_t)__popcll(peers));
        }
    } else if (kCount == 2) {
        ob.r[lane] = 0;
    }
}"""),
        NO_RANGE_CHECK,
    ],
    "pB": [
        ("""        const uint32_t h_l3 = tz_lds(w0, tbl) ^ tz_lds(w1, tbl + kTblWordsPerTupleWord);
        h = h_l3 ^ tz_lds(w2, tbl + 2 * kTblWordsPerTupleWord);""",
         """        const uint32_t h_l3 = w0 ^ (w1 * 0x9e3779b9u);   // MEASUREMENT: no table lookups
        h = h_l3 ^ (w2 * 0x85ebca6bu);"""),
    ],
    "pC": [
        ("""        const uint32_t rem = (P.mod_d & (P.mod_d - 1u)) == 0u
                                 ? h & (P.mod_d - 1u)
                                 : (uint32_t)__umul64hi(P.mod_m * (uint64_t)h, (uint64_t)P.mod_d);""",
         """        const uint32_t rem = h & (P.mod_d - 1u);   // MEASUREMENT: d a power of two only"""),
    ],
    "pD": [
        ("""        if (kCount == 2) {
            uint32_t before = 0;""",
         """        if (kCount == 2) {   // MEASUREMENT: counts only, no ranks (kCount 1's work)
            if (leader)
                atomicAdd(&cnt[bkt], (uint32_t)__popcll(peers));
            ob.r[lane] = 0;
        } else if (kCount == 5) {
            uint32_t before = 0;"""),
        NO_RANGE_CHECK,
    ],
    "grid1": [
        ("""        line_grid = std::max(1u, std::min(spans, resident_blocks(c, (const void *)line_fn,
                                                                 kLineBlock, lp.lds)));""",
         """        line_grid = std::max(1u, std::min(spans, resident_blocks(c, (const void *)line_fn,
                                                                 kLineBlock, lp.lds)));
        line_grid = std::min(line_grid, (uint32_t)c->cus);   // MEASUREMENT: one workgroup a CU"""),
    ],
    "pf2": [
        ("""    uint32_t tA = 0, sA = 0, tB = 0, sB = 0;
    if (slots_ok && tile_at(0, tA, sA)) {
        u32x4 rA[4], rB[4];
        uint32_t LA, LB;
        load_tile<true>(P, tA, P.n, lane, rA, LA);
        for (uint32_t i = 0;; i += 2) {
            const bool hB = tile_at(i + 1, tB, sB);
            load_tile<true>(P, hB ? tB : tA, P.n, lane, rB, LB);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sA * P.nb, slot(i), tA, P.n,
                                      lane, rA, LA);
            after(i, tA, !hB);
            if (!hB)
                break;
            const bool hA = tile_at(i + 2, tA, sA);
            load_tile<true>(P, hA ? tA : tB, P.n, lane, rA, LA);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sB * P.nb, slot(i + 1), tB,
                                      P.n, lane, rB, LB);
            after(i + 1, tB, !hA);
            if (!hA)
                break;
        }
    }""",
         """    uint32_t tA = 0, sA = 0, tB = 0, sB = 0, tC = 0, sC = 0;
    if (slots_ok && tile_at(0, tA, sA)) {
        // MEASUREMENT: two tiles of loads ahead (three register sets)
        u32x4 rA[4], rB[4], rC[4];
        uint32_t LA, LB, LC;
        load_tile<true>(P, tA, P.n, lane, rA, LA);
        bool hB = tile_at(1, tB, sB);
        load_tile<true>(P, hB ? tB : tA, P.n, lane, rB, LB);
        for (uint32_t i = 0;; i += 3) {
            const bool hC = hB && tile_at(i + 2, tC, sC);
            load_tile<true>(P, hC ? tC : hB ? tB : tA, P.n, lane, rC, LC);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sA * P.nb, slot(i), tA, P.n,
                                      lane, rA, LA);
            after(i, tA, !hB);
            if (!hB)
                break;
            const bool hA = hC && tile_at(i + 3, tA, sA);
            load_tile<true>(P, hA ? tA : hC ? tC : tB, P.n, lane, rA, LA);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sB * P.nb, slot(i + 1), tB,
                                      P.n, lane, rB, LB);
            after(i + 1, tB, !hC);
            if (!hC)
                break;
            hB = hA && tile_at(i + 4, tB, sB);
            load_tile<true>(P, hB ? tB : hA ? tA : tC, P.n, lane, rB, LB);
            process_tile<kC, kFilter>(P, tbl, kni, stage, cnt_w + sC * P.nb, slot(i + 2), tC,
                                      P.n, lane, rC, LC);
            after(i + 2, tC, !hA);
            if (!hA)
                break;
        }
    }"""),
    ],
}


def build(name: str) -> None:
    src = (CSRC / "yrss.hip").read_text()
    for anchor, repl in VARIANTS[name]:
        if src.count(anchor) != 1:
            raise SystemExit(f"{name}: anchor matches {src.count(anchor)} times: {anchor[:60]!r}")
        src = src.replace(anchor, repl)
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(CSRC / "yrss_line_prof.h", d)
        (Path(d) / "yrss.hip").write_text(src)
        out = ROOT / "ablib" / f"libyrss_{name}.so"
        out.parent.mkdir(exist_ok=True)
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-shared", "-Wall", "-Wno-unused-result", "-Wno-pass-failed",
               "-DYRSS_TOOLS_BUILD=1", "-I", str(ROOT / "include"), "-I", str(CSRC),
               str(Path(d) / "yrss.hip"), str(CSRC / "yrss_pcap.cpp"),
               str(CSRC / "yrss_shard.cpp"), str(CSRC / "yrss_fanout.cpp"), "-o", str(out)]
        subprocess.run(cmd, check=True)
    print(f"built {out.relative_to(ROOT)}")


if __name__ == "__main__":
    for v in sys.argv[1:] or sorted(VARIANTS):
        build(v)
