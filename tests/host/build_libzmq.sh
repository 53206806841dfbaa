#!/bin/sh
# Builds the CURVE interop test of config 1 (BASELINE.json configs[0]: CURVE
# PUSH/PULL over tcp://127.0.0.1, 1 KiB messages): two copies of the
# reference libzmq and the test program tests/host/test_curve_interop.cpp
# linked against each.
#   stock  the reference's src/*.cpp compiled where they lie under
#          /root/reference, CURVE over the image's libsodium 1.0.18
#          (/opt/conda), i.e. the reference's own codec;
#   zmqg   the same sources with INTEGRATION.md section 2 applied
#          (tests/host/libzmq_zmqg.patch, the ZMQ_USE_ZMQG_CURVE swap of
#          curve_encoding_t) in a scratch copy outside the repository, plus
#          libzmq_amd/host/curve_encoding_gpu.cpp, linked with
#          libzmq_amd/libzmqg_curve.so: the MESSAGE codec on the GPU, the
#          stream engine, I/O threads, handshake and sockets unchanged.
# The reference's own build system is not run: g++ on its sources with the
# test-only tests/host/ref_platform_full/platform.hpp in place of the
# generated one; the optional transports (WS, TIPC, VMCI, VSOCK, NORM, PGM)
# and GSSAPI are left out.  No reference source enters the repository;
# output only into tests/host/_ref/libzmq/ (git-ignored, travels to the GPU
# box, where /root/reference does not exist).  A no-op without the reference.
set -e
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT="$HERE/_ref/libzmq"
SODIUM=${SODIUM:-/opt/conda}
JOBS=${MAX_JOBS:-8}
[ -f "$REF/src/zmq.cpp" ] || { echo "build_libzmq: no reference sources at $REF; skipped"; exit 0; }
[ -f "$SODIUM/include/sodium.h" ] || { echo "build_libzmq: no libsodium at $SODIUM; skipped"; exit 0; }
mkdir -p "$OUT/stock/obj" "$OUT/zmqg/obj"

# the core library's sources (optional transports and GSSAPI left out)
list_sources () {
  for f in "$1"/src/*.cpp; do
    case $(basename "$f") in
      ws_*|wss_*|norm_*|pgm_*|tipc_*|vmci*|vsock_*|gssapi_*) ;;
      *) echo "$f" ;;
    esac
  done
}

CXXFLAGS="-O2 -std=c++11 -fPIC -D_REENTRANT -D_THREAD_SAFE"
export CXXFLAGS

# compile $2 (a source) into $1/obj with include flags $3
compile_all () {
  out=$1; src=$2; inc=$3
  list_sources "$src" | xargs -P "$JOBS" -I{} sh -c \
    'f={}; o='"$out"'/obj/$(basename $f .cpp).o; [ "$o" -nt "$f" ] || g++ $CXXFLAGS '"$inc"' -c "$f" -o "$o"'
}

# --- stock -----------------------------------------------------------------
INC_STOCK="-I$HERE/ref_platform_full -I$REF/include -I$REF/src -I$SODIUM/include"
compile_all "$OUT/stock" "$REF" "$INC_STOCK"
g++ -shared -o "$OUT/stock/libzmq.so.5" -Wl,-soname,libzmq.so.5 "$OUT"/stock/obj/*.o \
  "$SODIUM/lib/libsodium.so.23" -Wl,-rpath,"$SODIUM/lib" -lpthread

# --- zmqg: the patched copy, outside the repository -------------------------
SCRATCH=$(mktemp -d /tmp/zmqg_libzmq.XXXXXX)
trap 'rm -rf "$SCRATCH"' EXIT
cp -rp "$REF/src" "$REF/include" "$SCRATCH/"   # (times kept: up-to-date objects are reused)
patch -s -d "$SCRATCH" -p1 < "$HERE/libzmq_zmqg.patch"
# a changed source must rebuild (the patch touches two files; the class
# layout change reaches every file that includes them, so all are rebuilt
# when the patch or the adapter header is newer than the library)
if [ ! -f "$OUT/zmqg/libzmq.so.5" ] || [ "$HERE/libzmq_zmqg.patch" -nt "$OUT/zmqg/libzmq.so.5" ] \
   || [ "$ROOT/libzmq_amd/host/zmq_curve_encoding.hpp" -nt "$OUT/zmqg/libzmq.so.5" ] \
   || [ "$ROOT/libzmq_amd/host/curve_encoding_gpu.hpp" -nt "$OUT/zmqg/libzmq.so.5" ] \
   || [ "$ROOT/include/zmqg_curve.h" -nt "$OUT/zmqg/libzmq.so.5" ]; then
  rm -f "$OUT"/zmqg/obj/*.o
fi
INC_ZMQG="-DZMQ_USE_ZMQG_CURVE -I$HERE/ref_platform_full -I$SCRATCH/include -I$SCRATCH/src -I$SODIUM/include -I$ROOT/libzmq_amd/host"
compile_all "$OUT/zmqg" "$SCRATCH" "$INC_ZMQG"
g++ $CXXFLAGS -I"$ROOT/libzmq_amd/host" -c "$ROOT/libzmq_amd/host/curve_encoding_gpu.cpp" -o "$OUT/zmqg/obj/zmqg_curve_encoding_gpu.o"
g++ -shared -o "$OUT/zmqg/libzmq.so.5" -Wl,-soname,libzmq.so.5 "$OUT"/zmqg/obj/*.o \
  "$SODIUM/lib/libsodium.so.23" -Wl,-rpath,"$SODIUM/lib" \
  -L"$ROOT/libzmq_amd" -lzmqg_curve -Wl,-rpath,/root/repo/libzmq_amd -L/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -lpthread

# --- the test program, once per library (public zmq.h API only) -------------
for v in stock zmqg; do
  g++ -O2 -std=c++11 -Wall -Werror -I"$REF/include" -o "$OUT/interop_$v" "$HERE/test_curve_interop.cpp" \
    "$OUT/$v/libzmq.so.5" -Wl,-rpath,/root/repo/tests/host/_ref/libzmq/$v -lpthread
done
echo "build_libzmq: $OUT/interop_stock $OUT/interop_zmqg"
