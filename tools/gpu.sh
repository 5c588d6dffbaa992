#!/bin/bash
# tools/gpu.sh TAG 'STEP ARGS' ... -- the steps of one gpurun call, each under a
# time limit of its own, stopping at the first failure (no retries).  Output:
# gpurun_out/TAG/<i>_<kind>.{json,log,err} and a one-line summary per step.
#
#   tests [PYTEST ARGS]      pytest -m gpu over tests/ (e.g. "tests -k 'sample or c3'")
#   bench [BENCH ARGS]       python bench.py ARGS -> the JSON line, summarised
#   prof [BENCH ARGS]        rocprofv3 --kernel-trace --stats of bench.py --profile ARGS
#   pmc COUNTERS [ARGS]      one rocprofv3 --pmc pass (COUNTERS comma-free, '+'-joined)
#   traffic c2|c4 [ARGS]     FETCH_SIZE + WRITE_SIZE passes -> $O/pmc_<workload>.json
#   py SCRIPT [ARGS]         python SCRIPT ARGS
# A step may start with T=<seconds> (its time limit) and E=NAME=VALUE (an
# environment variable for that step only).
#
#   gpurun --timeout 900 -- tools/gpu.sh r5a 'tests -k sample' 'bench --gpus 2 --devices 0,0'
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for step in "$@"; do
    i=$((i + 1))
    lim=""
    envs=()
    while [[ $step == T=* || $step == E=* ]]; do
        w=${step%% *}; step=${step#* }
        if [[ $w == T=* ]]; then lim=${w#T=}; else envs+=("${w#E=}"); fi
    done
    for e in "${envs[@]}"; do export "$e"; done
    kind=${step%% *}
    args=""
    [[ $step == *" "* ]] && args=${step#* }
    base=$O/${i}_$kind
    eval "A=($args)"   # (quotes inside a step group words: "tests -k 'a or b'")
    echo "== step $i: $kind $args" | tee -a "$O/steps.txt"
    case $kind in
    tests)
        timeout -k 10 ${lim:-900} python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests "${A[@]}" \
            > $base.log 2>&1 || { tail -40 $base.log; exit 1; }
        tail -1 $base.log ;;
    bench)
        timeout -k 10 ${lim:-600} python -u bench.py "${A[@]}" > $base.json 2> $base.err || { tail -20 $base.err; exit 1; }
        python tools/summarize.py $base.json ;;
    prof)
        timeout -k 10 ${lim:-300} rocprofv3 --kernel-trace --stats -d $base.d -o kt --output-format csv -- \
            python3 bench.py --profile "${A[@]}" > $base.json 2> $base.err || { tail -20 $base.err; exit 1; }
        find $base.d -name '*kernel_stats.csv' -exec head -6 {} \; ;;
    pmc)
        ctr=${A[0]}
        timeout -s KILL ${lim:-120} rocprofv3 --pmc ${ctr//+/ } -d $base.d -o pmc --output-format csv -- \
            python3 bench.py --profile "${A[@]:1}" > $base.json 2> $base.err || { tail -20 $base.err; exit 1; }
        echo "pmc pass done: $ctr" ;;
    traffic)
        # HBM bytes per walk launch (roofline.traffic): FETCH_SIZE and WRITE_SIZE
        # in passes of their own, folded by pmc_summary.py into
        # $O/pmc_<workload>.json (copy to profiles/pmc_latest.json / pmc_c4.json)
        wl=${A[0]}; extra=("${A[@]:1}")
        sargs=(); [[ $wl == c4 ]] && sargs=(--workload C4 --filters 100000000)
        for pass in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL ${lim:-300} rocprofv3 --pmc $pass -d $base.d/$pass -o p --output-format csv -- \
                python3 bench.py --workload $wl --profile --steps 2 --warmup 1 "${extra[@]}" \
                > $base.$pass.json 2> $base.$pass.err || { tail -20 $base.$pass.err; exit 1; }
        done
        python3 tools/pmc_summary.py $base.d "${sargs[@]}" --write $O/pmc_$wl.json | tail -12 ;;
    py)
        timeout -k 10 ${lim:-600} python -u "${A[@]}" > $base.log 2> $base.err || { tail -20 $base.err; exit 1; }
        tail -5 $base.log ;;
    *)
        echo "unknown step kind: $kind"; exit 2 ;;
    esac
    for e in "${envs[@]}"; do unset "${e%%=*}"; done
done
echo DONE
