"""MI355X-native execution backend for the okapi-relational operator layer.

Drop-in replacement of the Flink backend of Cypher for Apache Flink for the
Table SPI (okapi-relational/.../api/table/Table.scala:43-178).  Layout:

  csrc/        HIP kernels (gfx950) + C++ runtime + the C-ABI (include/capf_gpu.h)
  _lib.py      ctypes binding of libcapf_gpu.so (fails loudly if not built)
  table.py     GpuSession / GpuTable — Table[GpuTable] over the C-ABI
  expr.py      Cypher IR subset + lowering to GPU expression programs
  header.py    RecordHeader (expr → column)
  graph.py     element tables + ScanGraph (label selection / alignment)
  planner.py   Expand / ExpandInto / var-length planning onto Table ops
  dist.py      one-process-per-GPU hash-partitioned 2-hop count (RCCL)

Import through capf_import.load() (the directory name is not a Python identifier).
"""
__all__ = ["table", "expr", "header", "graph", "planner"]
