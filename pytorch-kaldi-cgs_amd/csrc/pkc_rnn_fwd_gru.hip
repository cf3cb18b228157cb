// pkc_rnn_fwd_gru.hip — the forward time loops of the GRU, minimalGRU and RNN layers
// (kernels: pkc_rnn_impl.h)
#define PKC_RNN_FWD 1
#define PKC_RNN_PART 2
#include "pkc_rnn_impl.h"
