#!/bin/sh
# Builds the CURVE interop test of config 1 (BASELINE.json configs[0]: CURVE
# PUSH/PULL over tcp://127.0.0.1, 1 KiB messages): three copies of the
# reference libzmq and the test program tests/host/test_curve_interop.cpp
# linked against each.
#   stock  the reference's src/*.cpp, CURVE over the image's libsodium 1.0.18
#          (/opt/conda), i.e. the reference's own codec;
#   zmqg   the same sources with INTEGRATION.md section 2 applied
#          (tests/host/libzmq_zmqg.patch, the ZMQ_USE_ZMQG_CURVE swap of
#          curve_encoding_t) plus libzmq_amd/host/curve_encoding_gpu.cpp,
#          linked with libzmq_amd/libzmqg_curve.so: the MESSAGE codec on the
#          GPU, one device call per message, the stream engine, I/O threads,
#          handshake and sockets unchanged;
#   zmqgb  zmqg plus INTEGRATION.md section 3 (tests/host/libzmq_zmqg_batched.patch,
#          ZMQ_USE_ZMQG_CURVE_BATCHED): the stream engine hands its messages
#          to the I/O thread's batched codec (libzmq_amd/host/zmq_curve_engine.cpp,
#          curve_engine_hook.cpp, curve_batcher.cpp), whose eventfd sits in the
#          thread's poller.
# Every copy also carries tests/host/libzmq_test_switches.patch, test-only
# switches read from the environment (unset, the library behaves as the
# reference): ZMQG_TEST_ZMTP30 makes the side announce ZMTP 3.0, so its peer
# runs handshake_v3_0 with downgrade_sub (ZMQG_TEST_ZMTP30_TRACE reports it);
# INTEROP_PROFILE leaves SIGPROF unblocked in libzmq's threads for the test
# program's sampling profiler.
# The reference's own build system is not run: g++ on its sources, in scratch
# copies outside the repository, with the test-only
# tests/host/ref_platform_full/platform.hpp in place of the generated one;
# the optional transports (WS, TIPC, VMCI, VSOCK, NORM, PGM) and GSSAPI are
# left out.  No reference source enters the repository; output only into
# tests/host/_ref/libzmq/ (git-ignored, travels to the GPU box, where
# /root/reference does not exist).  A no-op without the reference.
set -e
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT="$HERE/_ref/libzmq"
SODIUM=${SODIUM:-/opt/conda}
JOBS=${MAX_JOBS:-8}
HOST="$ROOT/libzmq_amd/host"
[ -f "$REF/src/zmq.cpp" ] || { echo "build_libzmq: no reference sources at $REF; skipped"; exit 0; }
[ -f "$SODIUM/include/sodium.h" ] || { echo "build_libzmq: no libsodium at $SODIUM; skipped"; exit 0; }

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

SCRATCH=$(mktemp -d /tmp/zmqg_libzmq.XXXXXX)
trap 'rm -rf "$SCRATCH"' EXIT

# variant <name> <defines> <patches...>: a scratch copy of the reference with
# the patches applied, compiled into $OUT/<name>/libzmq.so.5.  All objects are
# rebuilt when a patch or a header of ours is newer than the library (a class
# layout change reaches every file that includes it); otherwise only sources
# newer than their objects.
variant () {
  name=$1; defs=$2; shift 2
  src="$SCRATCH/$name"
  mkdir -p "$src" "$OUT/$name/obj"
  cp -rp "$REF/src" "$REF/include" "$src/"   # (times kept: up-to-date objects are reused)
  stale=0
  [ -f "$OUT/$name/libzmq.so.5" ] || stale=1
  for p in "$@"; do
    patch -s -d "$src" -p1 < "$HERE/$p"
    [ "$HERE/$p" -nt "$OUT/$name/libzmq.so.5" ] && stale=1
  done
  if [ -n "$defs" ]; then
    for h in "$HOST"/*.hpp "$ROOT/include/zmqg_curve.h"; do
      [ "$h" -nt "$OUT/$name/libzmq.so.5" ] && stale=1
    done
  fi
  [ $stale = 1 ] && rm -f "$OUT/$name"/obj/*.o
  inc="$defs -I$HERE/ref_platform_full -I$src/include -I$src/src -I$SODIUM/include -I$HOST"
  list_sources "$src" | xargs -P "$JOBS" -I{} sh -c \
    'f={}; o='"$OUT/$name"'/obj/$(basename $f .cpp).o; [ "$o" -nt "$f" ] || g++ $CXXFLAGS '"$inc"' -c "$f" -o "$o"'
}

# link <name> <extra sources of ours...>
link () {
  name=$1; shift
  extra=""
  for f in "$@"; do
    o="$OUT/$name/obj/zmqg_$(basename "$f" .cpp).o"
    g++ $CXXFLAGS $inc -c "$HOST/$f" -o "$o"
    extra="$extra $o"
  done
  if [ -n "$extra" ]; then
    # libzmqg_curve.so found from the library's own place in the tree
    g++ -shared -o "$OUT/$name/libzmq.so.5" -Wl,-soname,libzmq.so.5 "$OUT/$name"/obj/*.o \
      "$SODIUM/lib/libsodium.so.23" -Wl,-rpath,"$SODIUM/lib" \
      -L"$ROOT/libzmq_amd" -lzmqg_curve -Wl,-rpath,'$ORIGIN/../../../../../libzmq_amd' \
      -L/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -lpthread
  else
    g++ -shared -o "$OUT/$name/libzmq.so.5" -Wl,-soname,libzmq.so.5 "$OUT/$name"/obj/*.o \
      "$SODIUM/lib/libsodium.so.23" -Wl,-rpath,"$SODIUM/lib" -lpthread
  fi
  # the test program (public zmq.h API only)
  g++ -O2 -std=c++11 -Wall -Werror -I"$REF/include" -o "$OUT/interop_$name" "$HERE/test_curve_interop.cpp" \
    "$OUT/$name/libzmq.so.5" -Wl,-rpath,'$ORIGIN/'"$name" -lpthread
}

variant stock "" libzmq_test_switches.patch
link stock
# the CPU baseline on the stock build's own curve_encoding_t (bench.py)
# (libsodium through a directory of its own: an rpath to $SODIUM/lib would
# also pick that tree's older libstdc++ for the program)
mkdir -p "$OUT/sodium" && ln -sf "$SODIUM/lib/libsodium.so.23" "$OUT/sodium/libsodium.so.23"
g++ $CXXFLAGS $inc -o "$OUT/curve_encoding_ref_bench" "$HERE/curve_encoding_ref_bench.cpp" \
  "$OUT/stock/libzmq.so.5" "$OUT/sodium/libsodium.so.23" -Wl,-rpath,'$ORIGIN/stock:$ORIGIN/sodium' -lpthread

variant zmqg "-DZMQ_USE_ZMQG_CURVE" libzmq_test_switches.patch libzmq_zmqg.patch
link zmqg curve_encoding_gpu.cpp

variant zmqgb "-DZMQ_USE_ZMQG_CURVE -DZMQ_USE_ZMQG_CURVE_BATCHED" \
  libzmq_test_switches.patch libzmq_zmqg.patch libzmq_zmqg_batched.patch
link zmqgb curve_encoding_gpu.cpp curve_batcher.cpp curve_engine_hook.cpp zmq_curve_engine.cpp

echo "build_libzmq: $OUT/interop_stock $OUT/interop_zmqg $OUT/interop_zmqgb"
