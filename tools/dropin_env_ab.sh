#!/bin/bash
# A/B of HIP runtime environment settings on the synchronous drop-in call
# (tools/dropin_bench, C2 stripe shape on device shards), two rounds
# interleaved; one JSON line per run on stdout, tagged with its setting.
set -o pipefail
run() {  # tag threads env...
        local tag=$1 th=$2; shift 2
        local out
        out=$(env "$@" timeout -k 10 60 tools/dropin_bench 10 4 1048576 64 "$th" 3 | grep '^{') || exit 1
        echo "{\"setting\": \"$tag\", \"threads\": $th, \"result\": $out}"
}
for round in 1 2; do
        for th in 1 16; do
                run default $th X=0 || exit 1
                run ROC_ACTIVE_WAIT_TIMEOUT=50 $th ROC_ACTIVE_WAIT_TIMEOUT=50 || exit 1
                run ROC_ACTIVE_WAIT_TIMEOUT=500 $th ROC_ACTIVE_WAIT_TIMEOUT=500 || exit 1
                run HIP_FORCE_DEV_KERNARG=0 $th HIP_FORCE_DEV_KERNARG=0 || exit 1
                run HIP_FORCE_DEV_KERNARG=0+WAIT50 $th HIP_FORCE_DEV_KERNARG=0 ROC_ACTIVE_WAIT_TIMEOUT=50 || exit 1
        done
done
