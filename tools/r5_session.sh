export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r5d.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_r5d.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/lanes_probe.py > gpurun_out/lanes_probe3.jsonl 2>gpurun_out/lanes_probe3.err || exit 1; cat gpurun_out/lanes_probe3.jsonl
tools/ab_prof.sh base ori || exit 1
python3 tools/ab_summary.py base ori
tools/ab_pmc_traffic.sh base ori || exit 1
echo ok
