"""dvcp -- MI355X-native (gfx950 HIP) DeepVCP registration hot path.

Drop-in for the reference's module surface (deepVCP.py, cpg.py, deep_feat_embedding.py,
deepVCP_loss.py, pointnet2_utils.py, voxelize.py, knn_cuda.KNN); see INTEGRATION.md.
"""
from ._lib import check_device_flags, load as load_library  # noqa: F401
from .cpg import cpg  # noqa: F401
from .deepVCP import DeepVCP  # noqa: F401
from .deepVCP_loss import deepVCP_loss, get_rigid_transform, svd_optimization  # noqa: F401
from .deep_feat_embedding import feat_embedding_layer  # noqa: F401
from .deep_feat_extraction import feat_extraction_layer  # noqa: F401
from .get_cat_feat_src import Get_Cat_Feat_Src  # noqa: F401
from .get_cat_feat_tgt import Get_Cat_Feat_Tgt  # noqa: F401
from .knn import KNN  # noqa: F401
from . import paper  # noqa: F401
# the reference harness's registration error (train.py:112-120, :156-164; C8 fixed): per pair on the
# GPU (dvcp_registration_error), so a multi-GPU job all-gathers it with the poses
from .ops import registration_error as registration_errors  # noqa: F401
from .datasets import KITTIDataset, ModelNet40Dataset  # noqa: F401
from .voxelize import voxelize, voxelize_point  # noqa: F401
from .weighting_layer import weighting_layer  # noqa: F401
