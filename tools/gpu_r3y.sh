export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/profile_r03.sh r03v3
