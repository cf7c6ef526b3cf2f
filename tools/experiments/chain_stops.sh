set -e
for v in "" chain_stop1 chain_stop2 no_chains; do
  KH_DEBUG=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify > gpurun_out/e_$v.log 2>&1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/e_$v.log') if l.startswith('{')][0]); print('$v', d['phases_ms'])"
done
