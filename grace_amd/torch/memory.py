"""``grace_dl.torch.memory.<name>`` -> the grace_amd.dist memories."""
import importlib
import sys

for _m in ("dgc", "efsignsgd", "none", "powersgd", "residual"):
    sys.modules[f"{__name__}.{_m}"] = importlib.import_module(f"grace_amd.dist.memory.{_m}")
