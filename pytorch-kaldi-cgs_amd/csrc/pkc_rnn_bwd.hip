// pkc_rnn_bwd.hip — the BPTT time loop of the recurrent layers (kernels: pkc_rnn_impl.h)
#define PKC_RNN_BWD 1
#include "pkc_rnn_impl.h"
