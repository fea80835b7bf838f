export TAG=${TAG:-pass} LIMIT=${LIMIT:-300} TAILN=${TAILN:-4}
bash tools/gpu_run.sh
