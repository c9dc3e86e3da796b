"""nerf_amd — MI355X (gfx950) NeRF ray-marching hot path behind the
sarphiv/nerf-experiments module API (positional_encodings, NerfModel,
NerfInterpolation).  See DESIGN.md at the repository root."""
from . import _lib, kernels  # noqa: F401
from .positional_encodings import (BarfPositionalEncoding, FourierFeatures, IdentityPositionalEncoding,  # noqa: F401
                                   IntegratedBarfFourierFeatures, IntegratedFourierFeatures, PositionalEncoding)
from .model_interpolation_architecture import NerfBaseModel, NerfModel  # noqa: F401
from .model_interpolation import MAGIC_NUMBER, NerfInterpolation, SchedulerLeNice  # noqa: F401
from .model_garf import GaussAct, ProposalNetwork, RadianceNetwork  # noqa: F401
from .model_ingp import INGPEncoding, INGPTable, NaiveINGP, NerfModelINGP  # noqa: F401
from .model_2d import FourierFeatures2d, Nerf2d  # noqa: F401
from .optim import FusedAdam  # noqa: F401
from .pose import compute_pose_error, kabsch_algorithm, validation_transform_rays  # noqa: F401
from .prop_sampler import PropNetEstimator, rendering  # noqa: F401

__version__ = "0.1.0"
