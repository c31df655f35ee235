# msm leg (tools/msm_ab.py) with the default library and every build_exp/ variant (GPU box)
OUT=gpurun_out/${1:-msmv}
mkdir -p $OUT
for lib in default build_exp/libnwcrypto_*.so; do
  name=$(basename $lib .so)
  if [ "$lib" = default ]; then
    timeout -k 10 180 python3 -u tools/msm_ab.py > $OUT/$name.jsonl 2>&1 || { echo "FAIL $name"; tail -5 $OUT/$name.jsonl; exit 1; }
  else
    NWCRYPTO_LIB=$PWD/$lib timeout -k 10 180 python3 -u tools/msm_ab.py > $OUT/$name.jsonl 2>&1 || { echo "FAIL $name"; tail -5 $OUT/$name.jsonl; exit 1; }
  fi
  echo "== $name"; cat $OUT/$name.jsonl
done
