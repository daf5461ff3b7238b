# Step time minus kernel time (the GPU-side gap between two frames' renders) for the product
# library against a baseline library (SVO_RT_LIB), interleaved, at the driver's K = 20 / W = 5
# and at K = 1000.  Baseline: build_ab/libsvo_rt_head.so (the sources of a git revision,
# built by hand with the flags of raytracingtest_amd/build.py).
#   bash tools/step_gap_ab.sh [rounds]
set -o pipefail
o=gpurun_out/step_gap; mkdir -p $o
for r in $(seq 1 ${1:-2}); do
  for lib in head product; do
    for kw in "20 5" "1000 200"; do
      set -- $kw
      if [ $lib = head ]; then export SVO_RT_LIB=$PWD/build_ab/libsvo_rt_head.so; else unset SVO_RT_LIB; fi
      timeout -k 10 180 python bench.py --no-extras --cpu-seconds 0 --steps $1 --warmup $2 > $o/$lib.$1.$r.json 2>$o/err.txt || exit $?
      python -c "import json;d=json.load(open('$o/$lib.$1.$r.json'));k=d['roofline']['kernel_ms'];print('$lib K=$1 round $r: step', d['ms_per_step'], 'kernel', k, 'gap_us', round((d['ms_per_step']-k)*1e3,2))"
    done
  done
done
