#!/bin/bash
# Builds the GeoFlink drop-in for libgeohip with one command (needs a JDK 8+ and the reference
# checked out and built once with `mvn -q -DskipTests package`; neither exists in this image):
#
#   REF=/path/to/SpatialFlink JAVA_HOME=/path/to/jdk jvm/build.sh
#
# Produces
#   jvm/lib/libgeohip_jni.so     the JNI shim (jvm/native/geohip_jni.c) linked to libgeohip.so
#   jvm/lib/geohip-geoflink.jar  GeoFlink.utils.GeoHip + GeoFlink.spatialOperators.geohip.*
# Use: put the jar on the job's classpath, run the JVM with -Djava.library.path=<repo>/jvm/lib,
# and construct GeoHipPointPointRangeQuery / GeoHipPointPointKNNQuery / GeoHipPointPointJoinQuery /
# GeoHipPointPolygonRangeQuery where the job constructed PointPointRangeQuery / PointPointKNNQuery /
# PointPointJoinQuery / PointPolygonRangeQuery (same constructor and run() arguments).
set -euo pipefail
cd "$(dirname "$0")/.."
: "${REF:?set REF to the reference checkout}"
: "${JAVA_HOME:?set JAVA_HOME to a JDK}"
python3 -m spatialflink_amd.build
mkdir -p jvm/lib jvm/classes
gcc -O2 -Wall -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -Iinclude jvm/native/geohip_jni.c \
    -Lspatialflink_amd -lgeohip -Wl,-rpath,"$PWD/spatialflink_amd" -o jvm/lib/libgeohip_jni.so
CP=$(cd "$REF" && mvn -q dependency:build-classpath -Dmdep.outputFile=/dev/stdout):$REF/target/classes
"$JAVA_HOME/bin/javac" -cp "$CP" -d jvm/classes $(find jvm/src -name '*.java')
"$JAVA_HOME/bin/jar" cf jvm/lib/geohip-geoflink.jar -C jvm/classes .
echo "built jvm/lib/libgeohip_jni.so jvm/lib/geohip-geoflink.jar"
