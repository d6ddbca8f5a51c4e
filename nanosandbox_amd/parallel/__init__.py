from .dist import (DistInfo, allreduce_sweep, destroy, init_distributed, node_rank_from_hostname, parse_transports,  # noqa: F401
                   rccl_env_defaults, report_transport, transport_kind)
from .reducer import FlatBucketReducer  # noqa: F401
