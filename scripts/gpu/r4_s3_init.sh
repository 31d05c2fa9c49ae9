#!/bin/bash
# first-call costs after HIP init: torch.manual_seed (seeds the GPU generators too),
# the CPU generator's manual_seed alone, and MnistNet() construction
set -o pipefail
mkdir -p gpurun_out/init
cat > gpurun_out/init/p2.py <<'PY'
import os, sys, time, json
sys.path.insert(0, os.getcwd())
import torch
from pytorch_operator_1_amd.models.mnist import MnistNet
order = sys.argv[1]
torch.zeros(1, device="cuda"); torch.cuda.synchronize()
out = {"order": order}
for step in order.split(","):
    t = time.time()
    if step == "seed":
        torch.manual_seed(1)
    elif step == "cpuseed":
        torch.default_generator.manual_seed(1)
    elif step == "net":
        MnistNet()
    elif step == "cudaseed":
        torch.cuda.manual_seed_all(1)
    out[step] = round(time.time() - t, 4)
print(json.dumps(out))
PY
for o in cpuseed,net,seed seed,net cudaseed,cpuseed,net; do
  timeout -k 10 120 python gpurun_out/init/p2.py $o >> gpurun_out/init/res2.jsonl || exit 1
done
cat gpurun_out/init/res2.jsonl
