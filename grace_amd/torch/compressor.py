"""``grace_dl.torch.compressor.<name>`` -> the grace_amd.dist compressors (identical codecs)."""
import importlib
import sys

for _m in ("dgc", "efsignsgd", "fp16", "natural", "none", "onebit", "powersgd", "qsgd", "randomk", "signsgd",
           "signum", "terngrad", "threshold", "topk"):
    sys.modules[f"{__name__}.{_m}"] = importlib.import_module(f"grace_amd.dist.compressor.{_m}")
