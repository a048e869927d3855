#!/bin/bash
# paged-layout LDS capacity sweep on the default C3 shard (documents per CU vs capacity failures)
set -u
mkdir -p gpurun_out
for c in "${@:-208,240,224}"; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --page-caps $c > gpurun_out/pcap_$c.json 2>gpurun_out/pcap_$c.err || { echo "caps $c failed"; tail -2 gpurun_out/pcap_$c.err; continue; }
  python -c "import json; d=json.load(open('gpurun_out/pcap_$c.json')); print('caps $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['paged_peaks'], d['parity']['replay_equals_generation'])"
done
