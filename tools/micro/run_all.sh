#!/bin/bash
for f in tools/micro/cemit_bench_*; do echo "== $f"; timeout -k 5 60 $f | head -1 || exit 1; done
