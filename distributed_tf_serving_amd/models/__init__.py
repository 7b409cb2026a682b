"""CTR model families (random-init; see ctr.py)."""
from .ctr import DCN, DLRM, FAMILIES, CTRModel, DCNv2, DeepFM, WideDeep, build_model  # noqa: F401
