#!/bin/bash
# Builds libkme_jni.so and GpuMatchingEngine.class (needs a JDK: JAVA_HOME, and the Kafka Streams
# jars plus the reference's compiled KProcessor on CLASSPATH for javac).
# Usage: bash integration/jni/build.sh [out_dir]
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=${1:-$HERE/out}
: "${JAVA_HOME:?JAVA_HOME must point at a JDK}"
mkdir -p "$OUT"
LIBDIR="$ROOT/kafka-matching-engine_amd/kme"
gcc -O2 -shared -fPIC -Wall -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I"$ROOT/include" \
    "$HERE/kme_jni.c" -L"$LIBDIR" -lkme -Wl,-rpath,"$LIBDIR" -o "$OUT/libkme_jni.so"
"$JAVA_HOME/bin/javac" -d "$OUT" "$HERE/GpuMatchingEngine.java"
echo "built $OUT/libkme_jni.so and $OUT/GpuMatchingEngine.class (run with -Djava.library.path=$OUT)"
