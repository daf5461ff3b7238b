set -o pipefail
o=gpurun_out/warm; mkdir -p $o
for w in 5 3000 5; do
  timeout -k 10 120 python bench.py --no-extras --cpu-seconds 0 --warmup $w --steps 50 > $o/w$w.json 2>$o/err.txt || exit $?
  python -c "import json,sys;d=json.load(open('$o/w$w.json'));print('warmup $w', d['ms_per_step'], d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else d['roofline'])"
done
timeout -k 10 120 python bench.py --no-extras --cpu-seconds 0 --warmup 3000 --steps 2000 > $o/long.json 2>>$o/err.txt || exit $?
python -c "import json;d=json.load(open('$o/long.json'));print('warm3000 steps2000', d['ms_per_step'])"
