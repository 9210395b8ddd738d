"""zasr — MI355X-native offline-ASR hot path (host package).

  zasr.model    Zipformer2 transducer config, synthetic weights, on-disk model format
  zasr.binding  ctypes binding of libzasr.so (the C ABI in include/zasr.h)
"""
