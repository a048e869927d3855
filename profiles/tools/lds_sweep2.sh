set -u
mkdir -p gpurun_out
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --steps 5 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || { echo "bench $tag failed"; tail gpurun_out/sw_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_$tag.json')); print('$tag', d['value'], d['roofline']['kernel_ms'], d['roofline']['docs_replayed_from_hbm']['total'], d['parity']['replay_equals_generation'])"
}
run o1000_c192 --ops 1000 --lds-cap 192
run o1000_c128 --ops 1000 --lds-cap 128
run o1000_c96 --ops 1000 --lds-cap 96
run o1000_c192_h96 --ops 1000 --lds-cap 192 --heap-cap 96
run o2000_c192_h96 --lds-cap 192 --heap-cap 96
run o2000_c160_h96 --lds-cap 160 --heap-cap 96
