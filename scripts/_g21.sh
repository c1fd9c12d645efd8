# GPU box: join_fused write pass with larger pair stages (768 per wave: 3 blocks per CU; 1024: 2)
# against the product (512, 4 blocks per CU) -- parity of the largest, then the join line per build.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g21
export TMPDIR=/tmp
CASES="product s640b768 s768b768 s896b768" WL=join STEPS=20 bash scripts/_lib_ab.sh
