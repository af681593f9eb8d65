set -o pipefail
mkdir -p gpurun_out/legs
timeout -k 10 300 python3 -c "
import sys; sys.path[:0]=['.','3d-mask-r-cnn_amd']
import torch, json, bench
from m3d.config import synthetic_rpn_config
from m3d.model import RPN, synthetic_volume
dev=torch.device('cuda')
m=RPN(synthetic_rpn_config(128),device=dev,seed=1)
with torch.no_grad(): f=m.features(synthetic_volume(128).to(dev))
print(json.dumps(bench.time_roi_align_bwd(f,128)))
print(json.dumps(bench.time_nms(dev)))
" > gpurun_out/legs/out.txt 2>&1; cat gpurun_out/legs/out.txt | grep -v amdgpu
