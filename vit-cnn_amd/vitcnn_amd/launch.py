"""Run the reference's own CLI (`main.py`) on the MI355X path, single-GPU or data parallel under torchrun.

    python -m vitcnn_amd.launch --main /path/to/reference/main.py [--precision fp32|bf16] -- <main.py args>
    torchrun --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 -m vitcnn_amd.launch \
        --main /path/to/reference/main.py -- --model Multimodality_Mamba --dataset Houston2013 ...

The reference's argparse (main.py:69-257) has no precision flag and no multi-process launch, and its
plugin import (main.py:46) names its own model_utils.  This shim reads main.py's text, applies the
edits below (each anchored on the exact reference line; a missing anchor raises, so a drifted
main.py is never run half-patched) and executes the result as `__main__`:

  * main.py:46   `from model_utils import get_model, train, test, pretrain` ->
                 the plugin surface from vitcnn_amd.model_utils (pretrain stays the reference's, raising when
                 called if the reference model_utils cannot be imported), and
                 `metrics` (main.py:505/514, utils.py:585-663) from vitcnn_amd.metrics;
  * main.py:52-53  stdout redirect: per-rank file name under data parallelism (`trytry.rank1.txt`);
  * main.py:257  `args = parser.parse_args()` -> `--precision` added (BASELINE config 2; it reaches
                 get_model through `hyperparams = vars(args)`, main.py:311), and the process group
                 initialised from torchrun's environment (`parallel.init_from_env`: RCCL, one GPU per
                 process; a no-op for one process);
  * main.py:259  `CUDA_DEVICE = get_device(args.cuda)` -> this rank's GPU (LOCAL_RANK) under DP.

train() (vitcnn_amd.model_utils) then shards the loader, exchanges gradients and keeps every rank's
control flow identical; only rank 0 writes checkpoints.  The patched text is also available without
running it (`patch_main_source`), which is what tests/test_launch_cpu.py checks.
"""
from __future__ import annotations

import argparse
import os
import sys

_EDITS = [
    ("from model_utils import get_model, train, test, pretrain",
     "try:\n"
     "    from model_utils import pretrain   # not on the ViT-CNN path (main.py calls it only with --pretrain)\n"
     "except Exception as _vc_e:   # the reference model_utils imports 15 modules absent from its tree\n"
     "    def pretrain(*_a, _err=repr(_vc_e), **_k):\n"
     "        raise RuntimeError('pretrain needs the reference model_utils, which does not import: ' + _err)\n"
     "from vitcnn_amd.model_utils import get_model, train, test\n"
     "from vitcnn_amd import parallel as _vc_parallel"),
    ("sys.stdout = open(filename, 'w')",
     "if int(os.environ.get('RANK', '0')) > 0:\n"
     "    filename = filename.replace('.txt', '.rank' + os.environ['RANK'] + '.txt')\n"
     "sys.stdout = open(filename, 'w')"),
    ("args = parser.parse_args()",
     "parser.add_argument('--precision', type=str, default='fp32', choices=['fp32', 'bf16'],\n"
     "                    help='GEMM operand precision of the MI355X ViT-CNN path (bf16: bf16 operands, fp32 accumulation)')\n"
     "args = parser.parse_args()\n"
     "_VC_RANK, _VC_WORLD, _VC_LOCAL = _vc_parallel.init_from_env()"),
    ("CUDA_DEVICE = get_device(args.cuda)",
     "CUDA_DEVICE = torch.device('cuda', _VC_LOCAL) if _VC_WORLD > 1 else get_device(args.cuda)"),
]
_METRICS_IMPORT = "from vitcnn_amd.metrics import metrics"


def patch_main_source(text: str) -> str:
    """main.py's text with the edits of the module docstring; raises RuntimeError on a missing anchor."""
    for anchor, repl in _EDITS:
        if text.count(anchor) != 1:
            raise RuntimeError(f"vitcnn_amd.launch: anchor not found exactly once in main.py: {anchor!r}")
        text = text.replace(anchor, repl)
    # utils.metrics -> the device confusion matrix (same result dict); imported after the reference's
    # own `from utils import ...` block so it takes precedence
    anchor = "from datasets import get_dataset"
    if text.count(anchor) != 1:
        raise RuntimeError(f"vitcnn_amd.launch: anchor not found exactly once in main.py: {anchor!r}")
    text = text.replace(anchor, "import os\n" + _METRICS_IMPORT + "\n" + anchor)
    return text


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(prog="python -m vitcnn_amd.launch")
    ap.add_argument("--main", required=True, help="path of the reference's main.py")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default=None,
                    help="shorthand for main.py's added --precision")
    a = ap.parse_args(argv)
    path = os.path.abspath(a.main)
    with open(path) as f:
        src = patch_main_source(f.read())
    if a.precision is not None:
        rest += ["--precision", a.precision]
    ref_dir = os.path.dirname(path)
    pkg_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (pkg_dir, ref_dir):
        if p not in sys.path:
            sys.path.insert(0, p)
    sys.argv = [path] + rest
    code = compile(src, path, "exec")
    glb = {"__name__": "__main__", "__file__": path}
    exec(code, glb)   # noqa: S102 -- the user's own main.py, patched as documented above


if __name__ == "__main__":
    main()
