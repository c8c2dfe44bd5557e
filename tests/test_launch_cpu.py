"""vitcnn_amd.launch: the reference CLI (main.py) patched for the MI355X path (VERDICT r2 missing item 2).

The patch is checked on the reference's own main.py text when the reference tree is present (the
build container; it is read as text and compiled, never executed -- it needs visdom and the .mat
datasets), and on a synthetic main.py carrying the same anchor lines everywhere else.
"""
import os

import pytest

REF_MAIN = "/root/reference/main.py"

SYNTH = """import torch
import sys
from utils import metrics, get_device
from datasets import get_dataset, MultiModalX
from model_utils import get_model, train, test, pretrain
import argparse
filename = './results/trytry.txt'
sys.stdout = open(filename, 'w')
parser = argparse.ArgumentParser()
parser.add_argument("--cuda", type=int, default=-1)
args = parser.parse_args()
CUDA_DEVICE = get_device(args.cuda)
hyperparams = vars(args)
"""


def _check(src):
    from vitcnn_amd.launch import patch_main_source
    out = patch_main_source(src)
    assert "from vitcnn_amd.model_utils import get_model, train, test" in out
    assert "from model_utils import get_model" not in out
    assert "    from model_utils import pretrain" in out
    assert "from vitcnn_amd.metrics import metrics" in out
    assert out.index("from vitcnn_amd.metrics import metrics") > out.index("from utils import")
    assert "'--precision'" in out and "_vc_parallel.init_from_env()" in out
    assert out.index("'--precision'") < out.index("args = parser.parse_args()")
    assert "torch.device('cuda', _VC_LOCAL) if _VC_WORLD > 1 else get_device(args.cuda)" in out
    assert ".rank' + os.environ['RANK']" in out
    compile(out, "main.py", "exec")
    return out


def test_patch_synthetic_main():
    _check(SYNTH)
    from vitcnn_amd.launch import patch_main_source
    with pytest.raises(RuntimeError, match="anchor"):
        patch_main_source(SYNTH.replace("args = parser.parse_args()", "args = parser.parse_known_args()[0]"))


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference tree absent (GPU box)")
def test_patch_reference_main():
    with open(REF_MAIN) as f:
        out = _check(f.read())
    # the argparse namespace feeds get_model through hyperparams = vars(args) (main.py:311)
    assert "hyperparams = vars(args)" in out
