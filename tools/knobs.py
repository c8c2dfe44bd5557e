"""Measurement switches for the tools: VITCNN_<NAME> environment variables -> the program's module constants.

The product package reads no environment (vitcnn_amd/model.py, fusatnet.py: module constants with the
measured-fastest defaults; the C ABI's kernel knobs exist only in libvitcnn_probe.so).  A tool that A/Bs
a switch (tools/ab_env.sh -> prof_step.py) imports this module first: it selects the probe library
and copies every VITCNN_* switch that is set onto the corresponding constant.
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
for _p in (_REPO, os.path.join(_REPO, "vit-cnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
PROBE_PATH = os.path.join(_REPO, "vit-cnn_amd", "vitcnn_amd", "libvitcnn_probe.so")
# the C ABI's kernel knobs (read by libvitcnn_probe.so only, common.h vc_knob)
PROBE_KNOBS = ("VITCNN_NL_LEGACY", "VITCNN_C2I_LDS", "VITCNN_TAP_NOSPLIT", "VITCNN_BN_PCAP", "VITCNN_BN_APPLY_ROWS", "VITCNN_BN_IM2COL",
               "VITCNN_BN_GLF", "VITCNN_SCAN_RBS", "VITCNN_SCAN_SELECT_RS", "VITCNN_SCAN_TAIL",
               "VITCNN_SPLITK_COMBINE", "VITCNN_LEGACY_COMBINE", "VITCNN_GEMM_PD", "VITCNN_GEMM_PIPE", "VITCNN_GEMM_PIPE_SMALL",
               "VITCNN_PIPE_NS", "VITCNN_PIPE_KS", "VITCNN_PIPE_BF_W8", "VITCNN_PIPE_F32_W8", "VITCNN_PIPE_SPLIT_BLOCKS", "VITCNN_PIPE_SPLIT_BELOW", "VITCNN_PIPE_SPLIT_FILL", "VITCNN_PIPE_KM", "VITCNN_GEMM_GROUP_MAXB",
               "VITCNN_TAP_TARGET", "VITCNN_TAP_PIPE", "VITCNN_CONV_PIPE_TILES_F", "VITCNN_CONV_PIPE_TILES_W",
               "VITCNN_CONV_PIPE_TILES_D", "VITCNN_CONV_PIPE_W8", "VITCNN_ATTN_BWD_WPB", "VITCNN_ATTN_FWD_WPB")


def use_probe():
    """bind lib() to libvitcnn_probe.so (call before the library is first used).  The product loader reads
    no environment; this tool-side switch honours VITCNN_LIB (an A/B build, tools/ab_steps.sh) or the probe."""
    from vitcnn_amd import _lib
    _lib.use_library_for_tools(os.environ.get("VITCNN_LIB", PROBE_PATH))


if "VITCNN_LIB" in os.environ or any(k in os.environ for k in PROBE_KNOBS):
    use_probe()

# env name -> (module, attribute, parser)
_FLAG = lambda v: v not in ("0", "", "false", "False")  # noqa: E731
SWITCHES = {
    "VITCNN_IMPLICIT_CONV": ("model", "_IMPLICIT_CONV", _FLAG),
    "VITCNN_DEFER_WGRAD": ("model", "_DEFER_WGRAD", _FLAG),
    "VITCNN_DEFER_WGRAD1": ("model", "_DEFER_WGRAD1", _FLAG),
    "VITCNN_SCAN_FUSED": ("model", "_SCAN_FUSED", _FLAG),
    "VITCNN_ROW_CHAIN": ("model", "_ROW_CHAIN", _FLAG),
    "VITCNN_GLF_FUSED": ("model", "_GLF_FUSED", _FLAG),
    "VITCNN_ONE_PARAM_REDUCE": ("model", "_ONE_PARAM_REDUCE", _FLAG),
    "VITCNN_TAP_DGRAD": ("model", "_TAP_DGRAD", _FLAG),
    "VITCNN_LANES": ("model", "_LANES", _FLAG),
    "VITCNN_LANES_BWD": ("model", "_LANES_BWD", _FLAG),
    "VITCNN_GEMM_GROUP": ("model", "_GROUP", _FLAG),
    "VITCNN_BF16_MIN_K": ("model", "_BF16_MIN_K", int),
    "VITCNN_GLOBAL_FIRST": ("model", "_GLOBAL_FIRST", _FLAG),
    "VITCNN_LANE_MAP": ("model", "_LANE_MAP", lambda v: [int(x) for x in v.split(",") if x]),
    "VITCNN_BN_TICKETS": ("model", "_BN_TICKETS", _FLAG),
    "VITCNN_BN_RELU_AFFINE": ("model", "_BN_RELU_AFFINE", _FLAG),
    "VITCNN_CH_LANE": ("model", "_CH_LANE", int),
    "VITCNN_CH_ORDERED": ("model", "_CH_ORDERED", _FLAG),
    "VITCNN_FUSAT_IM2COL": ("fusatnet", "_TAP_CONV", lambda v: not _FLAG(v)),
    "VITCNN_FUSAT_PAD_LIDAR": ("fusatnet", "_PAD_LIDAR", _FLAG),
    "VITCNN_GEMM_BNSTATS": ("model", "_GEMM_BNSTATS", _FLAG),
    "VITCNN_PG_LANE2": ("model", "_PG_LANE2", _FLAG),
}


def apply():
    import importlib
    done = {}
    for env, (mod, attr, parse) in SWITCHES.items():
        v = os.environ.get(env)
        if v is None:
            continue
        m = importlib.import_module("vitcnn_amd." + mod)
        setattr(m, attr, parse(v))
        done[env] = getattr(m, attr)
    if "VITCNN_IMPLICIT_CONV" in done:   # fusatnet imported the constant by value
        importlib.import_module("vitcnn_amd.fusatnet")._IMPLICIT_CONV = done["VITCNN_IMPLICIT_CONV"]
    return done


APPLIED = apply()
