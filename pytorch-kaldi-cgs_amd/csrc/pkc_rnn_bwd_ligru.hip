// pkc_rnn_bwd_ligru.hip — the BPTT time loop of the liGRU layers (kernels: pkc_rnn_impl.h)
#define PKC_RNN_BWD 1
#define PKC_RNN_PART 1
#include "pkc_rnn_impl.h"
