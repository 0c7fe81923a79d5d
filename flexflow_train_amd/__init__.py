"""flexflow_train_amd: an MI355X-native auto-parallelizing training framework
with FlexFlow-Train's capabilities (FFModel API, PCG IR, substitutions,
Unity / MCMC strategy search + simulator, RCCL-backed parallel execution).
"""
import torch  # noqa: F401  # load the HIP runtime before the native extensions

__version__ = "0.1.0"
