#!/bin/bash
# Paged LDS capacities 'pages,unsettled,heap' on C3 shard 0: which one moves the rate.
set -u
mkdir -p gpurun_out/caps_attr
for caps in 208,240,224 192,240,224 208,216,224 208,240,208 192,216,208 192,216,200; do
    timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 --shard 0 --page-caps $caps \
        > gpurun_out/caps_attr/$caps.json 2> gpurun_out/caps_attr/$caps.err || { tail -5 gpurun_out/caps_attr/$caps.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['roofline'].get('paged_caps'))" gpurun_out/caps_attr/$caps.json $caps
done
