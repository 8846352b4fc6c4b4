"""Diagnostics: run the CLI on test_cli_gpu.py::test_random_points_deterministic_with_debug's
config with HIP API logging (AMD_LOG_LEVEL=3) into gpurun_out/, under a hard time limit."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "fibsem-optflow_amd"))
import numpy as np
from PIL import Image
from optflow_amd import synth
out = ROOT / "gpurun_out" / "repro"
out.mkdir(parents=True, exist_ok=True)
I0, I1 = synth.gen_pair(150, 110, seed=41)
I1[:, :6] = 0
Image.fromarray(I0).save(out / "p.png")
Image.fromarray(I1).save(out / "q.png")
for k, debug in enumerate([False, True]):
    cfg = {"output_dir": str(out), "scale": 1, "output_type": "random_points",
           "npoints": 10, "debug": debug, "nscales": 3, "warps": 2, "rois": {"top": 30},
           "images": [{"p": str(out / "p.png"), "q": str(out / "q.png"),
                       "pId": "a", "qId": "b", "pGroupId": "1.0", "qGroupId": "2.0"}]}
    (out / f"cfg{k}.json").write_text(json.dumps(cfg))
    env = dict(os.environ, AMD_LOG_LEVEL="3")
    with open(out / f"log{k}.txt", "w") as f:
        try:
            r = subprocess.run([str(ROOT / "fibsem-optflow_amd/bin/optflow"), str(out / f"cfg{k}.json")],
                               stdout=f, stderr=subprocess.STDOUT, timeout=40, env=env)
            print(k, "rc", r.returncode, flush=True)
        except subprocess.TimeoutExpired:
            print(k, "TIMEOUT", flush=True)
