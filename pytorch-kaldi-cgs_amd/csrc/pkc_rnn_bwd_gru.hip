// pkc_rnn_bwd_gru.hip — the BPTT time loops of the GRU, minimalGRU and RNN layers
// (kernels: pkc_rnn_impl.h)
#define PKC_RNN_BWD 1
#define PKC_RNN_PART 2
#include "pkc_rnn_impl.h"
