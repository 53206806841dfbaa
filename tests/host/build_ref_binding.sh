#!/bin/sh
# Builds tests/host/_ref/test_zmq_binding_ref: the drop-in zmq::curve_encoding_t
# (libzmq_amd/host/zmq_curve_encoding.hpp) on the REFERENCE's own msg_t --
# src/msg.cpp, src/metadata.cpp and src/err.cpp compiled where they lie under
# /root/reference (nothing is copied), with the test-only
# tests/host/ref_platform/platform.hpp in place of the cmake-generated one.
# Output only into tests/host/_ref/ (git-ignored; it travels to the GPU box,
# where /root/reference does not exist).  Run by __graft_entry__.build() and
# tests/test_reference_binding.py; a no-op without the reference.
set -e
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT="$HERE/_ref"
[ -f "$REF/src/msg.cpp" ] || { echo "build_ref_binding: no reference sources at $REF; skipped"; exit 0; }
mkdir -p "$OUT"
INC="-I$HERE/ref_platform -I$REF/src -I$REF/include"
for f in msg metadata err; do
  g++ -O2 -std=c++11 -fPIC $INC -c "$REF/src/$f.cpp" -o "$OUT/ref_$f.o"
done
LIB="$ROOT/libzmq_amd"
g++ -O2 -std=c++11 -Wall -Werror -DZMQG_REAL_MSG_T=1 $INC -I"$ROOT/libzmq_amd/host" \
  -o "$OUT/test_zmq_binding_ref" "$HERE/test_zmq_binding.cpp" "$ROOT/libzmq_amd/host/curve_encoding_gpu.cpp" \
  "$OUT/ref_msg.o" "$OUT/ref_metadata.o" "$OUT/ref_err.o" \
  -L"$LIB" -lzmqg_curve -Wl,-rpath,"$LIB" -L/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -lpthread
echo "build_ref_binding: $OUT/test_zmq_binding_ref"
