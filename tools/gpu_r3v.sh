export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/demo_profile.py --steps 2 > gpurun_out/demo_prof.log 2>&1
echo "demo rc=$?"
