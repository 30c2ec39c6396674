"""nanotel_amd -- MI355X-native NanoTel hot path (HIP/gfx950) behind a C-ABI.

Mirrors the reference's per-chunk interface (NanoTel.R search_patterns /
analyze_read / run_future_worker_chuncks) on top of libnanotel.so.
"""
from ._lib import NanoTelError, lib, LIB_PATH  # noqa: F401
from .api import (NanoTel, assign_serials, read_blocks, synth_params, synth_read_ascii,  # noqa: F401
                  window_count, window_rows)

__version__ = "0.1.0"
