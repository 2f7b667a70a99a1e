#!/bin/bash
# A/B timing on the GPU box: tools/ab.sh "CFGS" spec... (spec = lib.so@ENC[:ENV=VAL,...])
cfgs=$1; shift
QB_CFG=$cfgs timeout -k 10 300 python tools/quick_bench.py "$@"
