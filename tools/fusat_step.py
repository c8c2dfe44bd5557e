"""GPU tool: bench.py's config-5 leg alone -- the FusAtNet B=64 training step as one hipGraph (and its
train-mode forward); prints the leg's JSON.  usage: python tools/fusat_step.py [steps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    out, _ = bench.fusat_leg(torch.device("cuda", 0), steps, False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
