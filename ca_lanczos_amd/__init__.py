"""ca_lanczos_amd -- MI355X-native CA-Lanczos hot path (HIP/gfx950 + RCCL).

Drop-in for the reference's hot-path functions (SpMV.m,
matrix_powers_{monomial,newton}.m, tsqr.m, cholqr.m, project.m,
normalize.m, projectAndNormalize.m, ca_lanczos.m, restarted_ca_lanczos.m,
impl_restarted_ca_lanczos.m) behind the C ABI of
include/calanczos.h; see DESIGN.md and INTEGRATION.md.
"""
from ._lib import CalError, LIB_PATH  # noqa: F401  (raises ImportError if the .so is missing)
from .api import (  # noqa: F401
    CALanczosOutput,
    Context,
    SpMV,
    ca_lanczos,
    ca_lanczos_ex,
    cholqr,
    compute_ritz_rnorm,
    context_for,
    default_context,
    eig,
    leja,
    matlab_rand,
    matrix_powers_monomial,
    matrix_powers_newton,
    newton_basis_matrix,
    normalize,
    project,
    projectAndNormalize,
    projectAndNormalize_ex,
    restarted_ca_lanczos,
    impl_restarted_ca_lanczos,
    tsqr,
)
from . import matrices  # noqa: F401
