#!/bin/sh
# ORACLE — TEST INFRASTRUCTURE ONLY.
#
# Compile the reference's own Toeplitz engine, KNI port-bitmap parser and INI
# reader from their source, where they lie, into oracle/_ref/libref_{thash,
# kni,ini}.so.  Two pieces of fs/lib/ff_dpdk_if.c need
# nothing beyond the C library and are compiled verbatim:
#   default_rsskey_40bytes   ff_dpdk_if.c:113-119
#   toeplitz_hash            ff_dpdk_if.c:1881-1902
# They are streamed into gcc on stdin (no source file is written anywhere), and
# two extern wrappers expose them.  toeplitz_dispatch itself is NOT built: it
# needs DPDK headers that require DPDK's generated rte_build_config.h, which
# the image lacks, so it is unbuildable here.
#
# Output: oracle/_ref/libref_thash.so (git-ignored, and listed in .gpurunignore:
# no reference-compiled object goes to the GPU box).
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${YRSS_REFERENCE:-/root/reference}
SRC="$REF/fs/lib/ff_dpdk_if.c"
if [ ! -f "$SRC" ]; then
    echo "build_ref.sh: $SRC not present; oracle/_ref not built" >&2
    exit 0
fi
mkdir -p "$HERE/_ref"
{
    printf '#include <stdint.h>\n#include <sys/types.h>\n'
    printf '#line 1 "%s"\n' "$SRC"
    awk '/^static uint8_t default_rsskey_40bytes/ {f = 1} f {print} f && /^};/ {exit}' "$SRC"
    awk 'prev ~ /^static uint32_t[ \t]*$/ && /^toeplitz_hash\(/ {print prev; f = 1}
         f {print}
         f && /^}/ {exit}
         {prev = $0}' "$SRC"
    cat <<'EOF'
uint32_t ref_toeplitz_hash(unsigned keylen, const uint8_t *key,
                           unsigned datalen, const uint8_t *data)
{ return toeplitz_hash(keylen, key, datalen, data); }
const uint8_t *ref_default_rsskey(void) { return default_rsskey_40bytes; }
/* timing loop for the CPU-baseline calibration (DESIGN.md §6) */
uint32_t ref_bench_hash(const uint8_t *tuples, unsigned n, unsigned reps)
{
    uint32_t acc = 0;
    for (unsigned r = 0; r < reps; ++r)
        for (unsigned i = 0; i < n; ++i)
            acc += toeplitz_hash(40, default_rsskey_40bytes, 12, tuples + 12 * i);
    return acc;
}
EOF
} | ${CC:-gcc} -O2 -frename-registers -funswitch-loops -fweb -fPIC -shared -x c - \
      -o "$HERE/_ref/libref_thash.so"
echo "build_ref.sh: built $HERE/_ref/libref_thash.so"

# The INI reader fs/lib vendors (inih, fs/lib/ff_ini_parser.c + .h) is plain
# C: compiled where it lies into oracle/_ref/libref_ini.so, the checker of
# yastack_amd/ffconfig.py's reader (tests/test_ffconfig.py).
INI="$REF/fs/lib/ff_ini_parser.c"
if [ -f "$INI" ]; then
    ${CC:-gcc} -O2 -fPIC -shared "$INI" -o "$HERE/_ref/libref_ini.so"
    echo "build_ref.sh: built $HERE/_ref/libref_ini.so"
fi

# The KNI port bitmaps, fs/lib/ff_dpdk_kni.c: the bit macros and magic_bits
# (:51-58), set_bitmap / get_bitmap (:83-96) and kni_set_bitmap (:98-123) need
# only htons, strstr and atoi, so they too are compiled verbatim, streamed
# from the reference file into gcc, into oracle/_ref/libref_kni.so.
KNI="$REF/fs/lib/ff_dpdk_kni.c"
if [ ! -f "$KNI" ]; then
    echo "build_ref.sh: $KNI not present; libref_kni.so not built" >&2
    exit 0
fi
{
    printf '#include <stdint.h>\n#include <stdlib.h>\n#include <string.h>\n#include <arpa/inet.h>\n'
    printf '#line 1 "%s"\n' "$KNI"
    awk '/^#define (set|clear|get)_bit\(/ {print}' "$KNI"
    awk '/^static const int magic_bits/ {f = 1} f {print} f && /^};/ {exit}' "$KNI"
    for fn in set_bitmap get_bitmap kni_set_bitmap; do
        awk -v fn="$fn" 'prev ~ /^static (void|int)[ \t]*$/ && index($0, fn "(") == 1 {print prev; f = 1}
             f {print}
             f && /^}/ {exit}
             {prev = $0}' "$KNI"
    done
    cat <<'EOF2'
void ref_kni_set_bitmap(const char *p, unsigned char *bm) { kni_set_bitmap(p, bm); }
int ref_get_bitmap(uint16_t port, unsigned char *bm) { return get_bitmap(port, bm); }
void ref_set_bitmap(uint16_t port, unsigned char *bm) { set_bitmap(port, bm); }
EOF2
} | ${CC:-gcc} -O2 -fPIC -shared -x c - -o "$HERE/_ref/libref_kni.so"
echo "build_ref.sh: built $HERE/_ref/libref_kni.so"
