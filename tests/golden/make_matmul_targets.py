"""tests/golden/matmul_targets.json: the reference's fault-campaign target files
(input/{encoder,decoder}/matmul_*.json: target MatMul, its input / weight / output tensor
names in the exported graphs), collected as data (build container only):

    python tests/golden/make_matmul_targets.py
"""
import glob
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("QTX_REFERENCE", "/root/reference")

out = []
for mod in ("encoder", "decoder"):
    for p in sorted(glob.glob(os.path.join(REF, "input", mod, "matmul_*.json"))):
        j = json.load(open(p))
        out.append({k: j[k] for k in ("target_layer", "input_tensor", "weight_tensor",
                                      "output_tensor", "module")})
json.dump(out, open(os.path.join(HERE, "matmul_targets.json"), "w"), indent=1)
print(len(out), "targets")
