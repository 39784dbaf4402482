set -o pipefail
mkdir -p gpurun_out/c2
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/c2/$name.log 2>&1; local rc=$?; tail -30 gpurun_out/c2/$name.log; echo "== $name rc=$rc"; return $rc; }
run gpuinfo 60 ./kgs/_native/kgs-gpuinfo && \
run gpuinfo_json 60 ./kgs/_native/kgs-gpuinfo --json && \
run dp_selftest 120 python -m kgs.deviceplugin --self-test && \
run entrypoint 600 python -m kgs.workload.entrypoint --gemm-size 8192 --json-out gpurun_out/c2/entry.json
