// pkc_rnn_fwd_ligru.hip — the forward time loop of the liGRU layers (kernels: pkc_rnn_impl.h)
#define PKC_RNN_FWD 1
#define PKC_RNN_PART 1
#include "pkc_rnn_impl.h"
