# stats sweep A/B on the headline bench (interleaved, 3 rounds)
for r in 1 2 3; do
for v in "1 512" "1 256" "1 384" "1 640"; do
  set -- $v
  printf "tile=%s grid=%s " $1 $2
  SMQ_STATS_TILE=$1 SMQ_STATS_GRID=$2 timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
SMQ_STATS_TILE=1 SMQ_STATS_GRID=256 bash tools/ktrace.sh stx_256 smaq 30 | grep -E "stats|apply" | cut -c1-160
SMQ_STATS_TILE=1 SMQ_STATS_GRID=512 bash tools/ktrace.sh stx_512 smaq 30 | grep -E "stats|apply" | cut -c1-160
