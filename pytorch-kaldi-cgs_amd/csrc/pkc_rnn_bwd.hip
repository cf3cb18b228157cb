// pkc_rnn_bwd.hip — the BPTT time loop of the LSTM layers and the pkc_rnn_bwd dispatch
// (kernels: pkc_rnn_impl.h; liGRU: pkc_rnn_bwd_ligru.hip, GRU / minimalGRU / RNN: pkc_rnn_bwd_gru.hip)
#define PKC_RNN_BWD 1
#define PKC_RNN_PART 0
#include "pkc_rnn_impl.h"
