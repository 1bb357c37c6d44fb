# The round-6 forward wave-count rule (7 / 8 / 4 waves by groups per CU) at HEAD: same-box
# A/B against the previous counts (6 up to 2,048 groups, 4 beyond), the GPU tests and the
# driver-form bench line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=512,2048,8192,16384,65536" plan= ns6=LV_TILE_NSEG=6 ns4=LV_TILE_NSEG=4 plan2= ns6b=LV_TILE_NSEG=6 > gpurun_out/ab_nseg_rule.log 2>&1 || { echo ab failed; cat gpurun_out/ab_nseg_rule.log; exit 1; }
cat gpurun_out/ab_nseg_rule.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nseg_pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/nseg_pytest.log; exit 1; }
tail -n 2 gpurun_out/nseg_pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/nseg_bench.log 2>&1 || { echo bench failed; tail gpurun_out/nseg_bench.log; exit 1; }
tail -n 1 gpurun_out/nseg_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'us', d['roofline']['us_per_launch_events'], 'frac', d['roofline']['frac'], 'sweep', d['sweep'], 'c5', d['config5']['us_per_launch'], 'train', {k: d['train_step'][k]['ms_per_step'] for k in ('f32','bf16')}, 'fwd_bwd', d['fwd_bwd']['us_per_step'])"
