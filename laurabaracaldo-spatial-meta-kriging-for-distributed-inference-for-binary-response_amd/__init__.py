"""MI355X-native spatial meta-kriging for binary responses (drop-in for the
data-parallel core of MetaKriging_BinaryResponse.R).

The compute path is libmk.so (HIP, gfx950) behind the C ABI in include/mk.h;
this package is the host-side mirror of the reference's R interface
(spMvGLM / spPredict / partitioned_spMvGLM / the combine) over ctypes.
"""
from ._lib import MkError, load  # noqa: F401
from .session import SamplerConfig, Session, cholesky_batched, combine, correlation_batched  # noqa: F401
from .spbayes import spMvGLM, spPredict  # noqa: F401
from .glm import glm_binomial  # noqa: F401
from .post import combine_median  # noqa: F401
from .metakriging import (combine_results, meta_fit, partition, partitioned_spMvGLM,  # noqa: F401
                          posterior_summary, start_values, subset_data)
from .node import meta_fit_node  # noqa: F401
from . import synthetic  # noqa: F401
