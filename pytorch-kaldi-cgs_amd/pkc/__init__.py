"""pkc — MI355X-native hot path of pytorch-kaldi-CGS's run_nn() (chunk training loop).

Modules:
  pkc.neural_networks  drop-in arch plug-ins (arch_library = pkc.neural_networks)
  pkc.core             drop-in run_nn (same signature / return value / side files)
  pkc.engine           executor of the [model] graph on libpkc.so HIP kernels
  pkc.data_io          Kaldi ark I/O + GPU chunk preparation
  pkc._lib             ctypes binding of libpkc.so (C ABI: include/pkc.h)
"""
__version__ = "0.1.0"
