"""fury_amd — MI355X-native bulk encoder/decoder for Apache Fory's row format.

Scope: the java/fory-format row-format path only. The compute
lives in hand-written gfx950 HIP kernels behind the C-ABI in
include/fory_rowfmt.h (fury_amd/lib/libfory_rowfmt.so).
"""
__version__ = "0.1.0"
