set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_za
for rep in 1 2 3; do
for c in 0 1; do
  GSGPU_YOUNG_COMBINE=$c timeout -k 10 200 python -u tools/window_profile.py 12 > gpurun_out/r06_za/wp_c${c}_$rep.txt 2> gpurun_out/r06_za/wp_c${c}_$rep.err || { echo WP_FAIL; tail -5 gpurun_out/r06_za/wp_c${c}_$rep.err; exit 1; }
  echo "c=$c rep=$rep $(head -1 gpurun_out/r06_za/wp_c${c}_$rep.txt) | $(tail -1 gpurun_out/r06_za/wp_c${c}_$rep.txt)"
done
done
for c in 0 1; do
  GSGPU_YOUNG_COMBINE=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/r06_za/bench_c$c.json 2> gpurun_out/r06_za/bench_c$c.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r06_za/bench_c$c.json'));print('bench c=$c', d['ms_per_step'], d['final_checksum_vs_fixture']['match'])"
done
