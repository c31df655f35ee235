set -o pipefail
OUT=gpurun_out/${1:-r04n}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u tools/worker_probe.py > $OUT/worker_probe.jsonl 2> $OUT/worker_probe.err || { echo "PROBE FAILED"; tail -20 $OUT/worker_probe.err; exit 1; }
cat $OUT/worker_probe.jsonl
timeout -k 10 200 python3 -u bench.py --streams 1 --no-extras --no-cpu-baseline --latency-samples 0 > $OUT/bench_s1.json 2> $OUT/bench_s1.err || { echo "BENCH S1 FAILED"; tail -20 $OUT/bench_s1.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --streams 2 --no-extras --no-cpu-baseline --latency-samples 0 > $OUT/bench_s2.json 2> $OUT/bench_s2.err || { echo "BENCH S2 FAILED"; tail -20 $OUT/bench_s2.err; exit 1; }
for f in s1 s2; do python3 -c "import json; d=json.loads(open('$OUT/bench_$f.json').read().strip().splitlines()[-1]); print('C2 $f', d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"; done
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('C2', d['value']/1e6, d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['worker_digest'])[:700])"
timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('C4 default', d['value']/1e6, d['ms_per_step'])"
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_prio.so timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_prio.json 2> $OUT/bench_c4_prio.err || { echo "C4 PRIO FAILED"; tail -20 $OUT/bench_c4_prio.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4_prio.json').read().strip().splitlines()[-1]); print('C4 prio', d['value']/1e6, d['ms_per_step'])"
timeout -k 10 400 python3 -u tools/bench_configs.py --only C3,C5 --cpu-seconds 0 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "CONFIGS FAILED"; tail -20 $OUT/configs.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); print(d['config'], round(d['sigs_per_s']/1e6,1), round(d['ms_per_step'],3), 'serial', round(d['sigs_per_s_serial']/1e6,1), d['parity'])"
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_prio.so timeout -k 10 400 python3 -u tools/bench_configs.py --only C5 --cpu-seconds 0 > $OUT/configs_prio.jsonl 2> $OUT/configs_prio.err || { echo "CONFIGS PRIO FAILED"; tail -20 $OUT/configs_prio.err; exit 1; }
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_prio.so timeout -k 10 200 python3 -u bench.py --streams 2 --no-extras --no-cpu-baseline --latency-samples 0 > $OUT/bench_s2_prio.json 2> $OUT/bench_s2_prio.err || { echo "BENCH S2 PRIO FAILED"; tail -20 $OUT/bench_s2_prio.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs_prio.jsonl'):
    d=json.loads(l); print('prio', d['config'], round(d['sigs_per_s']/1e6,1), round(d['ms_per_step'],3), 'serial', round(d['sigs_per_s_serial']/1e6,1), d['parity'])
d=json.loads(open('$OUT/bench_s2_prio.json').read().strip().splitlines()[-1]); print('C2 s2 prio', d['value']/1e6, d['ms_per_step'])"
exit 0
