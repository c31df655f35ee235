set -o pipefail
OUT=gpurun_out/${1:-r04j}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep -E '"x_mode": (0|7)' $OUT/sha_lone.jsonl | cut -c1-200
for k in 1 2; do
timeout -k 10 300 python3 -u tools/host_fed_reps.py 30 > $OUT/host_fed_gc$k.json 2> $OUT/host_fed_gc$k.err || { echo "HOSTFED FAILED"; tail -5 $OUT/host_fed_gc$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/host_fed_gc$k.json')); print('gc on ', round(d['median_ms'],3), [round(p['ms'],2) for p in d['passes']], 'fresh', [round(x,2) for x in d['fresh_passes_ms']])"
timeout -k 10 300 python3 -u tools/host_fed_reps.py 30 nogc > $OUT/host_fed_nogc$k.json 2> $OUT/host_fed_nogc$k.err || { echo "HOSTFED FAILED"; tail -5 $OUT/host_fed_nogc$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/host_fed_nogc$k.json')); print('gc off', round(d['median_ms'],3), [round(p['ms'],2) for p in d['passes']], 'fresh', [round(x,2) for x in d['fresh_passes_ms']])"
done
exit 0
