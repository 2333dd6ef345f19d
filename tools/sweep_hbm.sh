set -e
for nb in 128 256 512 1024 2048; do echo "BN_BLOCKS=$nb"; S3OD_BN_BLOCKS=$nb timeout -k 5 60 python -c "
import sys; sys.path.insert(0,'.'); from tools.hbm_bench import bn_bwd; bn_bwd(relu=True); bn_bwd(relu=False)" 2>&1 | grep -v amdgpu; done
for r in 16 32 64 128 256; do echo "UNROPE_RPB=$r"; S3OD_UNROPE_RPB=$r timeout -k 5 60 python -c "
import sys; sys.path.insert(0,'.'); from tools.hbm_bench import unrope; unrope()" 2>&1 | grep -v amdgpu; done
