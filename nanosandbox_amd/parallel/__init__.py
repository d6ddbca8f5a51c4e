from .dist import DistInfo, destroy, init_distributed, node_rank_from_hostname, rccl_env_defaults  # noqa: F401
from .reducer import FlatBucketReducer  # noqa: F401
