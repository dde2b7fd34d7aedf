for c in 0 256 128 64 0 256 128; do
  timeout -k 10 200 python bench.py --scene synthetic:10000 --steps 2 --warmup 1 --cpu-baseline off --chunk $c > gpurun_out/c5chunk_$c.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c5chunk_$c.json'));print('chunk $c', d['ms_per_step'])"
done
