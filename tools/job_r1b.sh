#!/bin/bash
source ./gpurun_job.sh
export TMPDIR=/tmp
step pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
bash tools/job_prof.sh
