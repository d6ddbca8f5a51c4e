from .loader import (  # noqa: F401
    MemmapBatchSource,
    NativeBatchSource,
    SyntheticBatchSource,
    load_meta,
    make_batch_source,
    resolve_data_dir,
)
