// pkc_rnn_fwd.hip — the forward time loop of the LSTM layers and the pkc_rnn_fwd dispatch
// (kernels: pkc_rnn_impl.h; liGRU: pkc_rnn_fwd_ligru.hip, GRU / minimalGRU / RNN: pkc_rnn_fwd_gru.hip)
#define PKC_RNN_FWD 1
#define PKC_RNN_PART 0
#include "pkc_rnn_impl.h"
