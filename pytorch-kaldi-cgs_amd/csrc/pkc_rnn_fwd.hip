// pkc_rnn_fwd.hip — the forward time loop of the recurrent layers (kernels: pkc_rnn_impl.h)
#define PKC_RNN_FWD 1
#include "pkc_rnn_impl.h"
