#!/bin/sh
# Sampling profile of both I/O threads of one CURVE PUSH/PULL pair
# (tests/host/test_curve_interop.cpp, INTEROP_PROFILE): usage
#   tools/profile_pair.sh <server kind> <client kind> <out prefix> [messages]
# writes <out prefix>.pull.err / .push.err (prof / cpu / zmqg engine lines).
set -e
B=$(cd "$(dirname "$0")/.." && pwd)/tests/host/_ref/libzmq
S=$1; C=$2; O=$3; N=${4:-1000000}
P=$(python3 -c 'import socket;s=socket.socket();s.bind(("127.0.0.1",0));print(s.getsockname()[1])')
Q=$((P + 1))
export INTEROP_THREAD_CPU=1 ZMQG_ENGINE_STATS=1
[ -n "$NOPROF" ] || export INTEROP_PROFILE=1
"$B/interop_$S" pull tcp://127.0.0.1:$P tcp://127.0.0.1:$Q $N 11 5 > "$O.pull.out" 2> "$O.pull.err" &
PID=$!
sleep 0.5
"$B/interop_$C" push tcp://127.0.0.1:$P tcp://127.0.0.1:$Q $N 11 5 > "$O.push.out" 2> "$O.push.err"
wait $PID
cat "$O.pull.out"
