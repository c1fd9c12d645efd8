#!/bin/bash
# Before every gpurun: rebuild the library (and the oracle, the JNI test shim) from the current
# sources and run the CPU suite, so the snapshot never carries a stale libgeohip.so.
set -e
cd "$(dirname "$0")/.."
python3 __graft_entry__.py > /tmp/preflight_build.log 2>&1 || { tail -20 /tmp/preflight_build.log; exit 1; }
python3 -m pytest tests -q -m "not gpu" -x -n 8 2>&1 | tail -1
