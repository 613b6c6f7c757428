#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE + WRITE_SIZE passes (each its own run, as
# MI355X_MICROARCH.md's HBM section prescribes) of the join alone, T = 64 and T = 128;
# summaries into gpurun_out/pmc/*.json (copy into profiles/ to keep them)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
run() {   # name k replicas
    local n=$1 k=$2 r=$3
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$n.stats -o run --output-format csv -- \
        python3 tools/join_probe.py --k $k --replicas $r > $O/$n.stats.log 2>&1 || return 1
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$n.fetch -o run --output-format csv -- \
        python3 tools/join_probe.py --k $k --replicas $r > $O/$n.fetch.log 2>&1 || return 1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/$n.write -o run --output-format csv -- \
        python3 tools/join_probe.py --k $k --replicas $r > $O/$n.write.log 2>&1 || return 1
    python3 tools/pmc_summary.py --stats-dir $O/$n.stats --fetch-dir $O/$n.fetch \
        --write-dir $O/$n.write --kernel "k_or16<2" --replicas $r --pairs $k --out $O/$n.json
}
run join_t64 1 1048576 && run join_t128 2 524288
