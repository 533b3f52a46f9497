#!/bin/bash
# round 5: step suite with the mixed-precision Newton refinement + stage profile, then the fused TQC
# learner tests, then the bench
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r5t}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --deselect tests/test_tqc_gpu.py > $OUT/${TAG}_pytest.log 2>&1
rc=$?; tail -4 $OUT/${TAG}_pytest.log; grep -E "^FAILED|worst error / bar \[" $OUT/${TAG}_pytest.log | cut -c1-200 | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/step_parity.py 4096 prof bench > $OUT/${TAG}_stageprof.log 2>&1 || exit $?
grep -E "M env|per env|newton|n_newton|noslip " $OUT/${TAG}_stageprof.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_tqc_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread > $OUT/${TAG}_tqc.log 2>&1
rc=$?; tail -4 $OUT/${TAG}_tqc.log; grep -E "fused|learner step|logs|Error|assert" $OUT/${TAG}_tqc.log | cut -c1-400 | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/${TAG}_bench.log 2>&1 || exit $?
tail -1 $OUT/${TAG}_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('C3', r['value'], 'kernel ms', r['roofline']['kernel_avg_ms']); print('gym', r['gym']['gym_steps_per_s']); print('tqc', {k: r['tqc'][k] for k in ('gym_steps_per_s','learner_ms_per_update','transitions_per_s_at_reference_utd','learner')}); print('ik', r.get('ik', {}).get('value'))"
