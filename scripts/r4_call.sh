# one gpurun call: each GPU step under its own time limit; stop at the first
# step that faulted, aborted or hit its limit (plain test failures go on)
set -o pipefail
mkdir -p gpurun_out
step() {   # step <name> <limit-seconds> <log> <command...>
    local name=$1 lim=$2 log=$3; shift 3
    echo "== $name" >> gpurun_out/steps.txt
    timeout -k 10 "$lim" "$@" > "$log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >> gpurun_out/steps.txt
    if grep -q -i -E "illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|no GPU 0 visible" "$log"; then
        echo "== $name: GPU fault seen, stopping" >> gpurun_out/steps.txt; exit 99
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name (rc=$rc)"; exit $rc; fi
    return 0
}
