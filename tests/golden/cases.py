"""Configurations shared by the golden generator (make_golden.py) and the parity tests.

Option names and values follow the reference's cfg schema (proto/MLP.proto, proto/liGRU.proto,
proto/LSTM.proto plus the CGS keys read at neural_networks.py:98-131, 490-529).
"""
import configparser
import os

_TMP = "/tmp"

MLP_DEF = dict(dnn_drop="0.0", dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False",
               dnn_use_batchnorm="True", dnn_use_laynorm="False", dnn_act="relu", to_do="train",
               mlp_hcgs="False", hcgs_block="16,4", hcgs_sparse="50,50", out_folder=_TMP,
               mlp_quant="False", param_quant="8", mlp_quant_inp="False", inp_quant="16",
               mlp_prune="False", mlp_prune_perc="70", skip_regularization="True",
               guided_hcgs="False", apply_guided_hcgs="False", arch_name="MLP_layers1",
               use_cuda="False")



def build_mlp_config(variant):
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"use_cuda": "False", "to_do": "train", "seed": "2234"}
    body = dict(MLP_DEF, arch_name="MLP_layers1", dnn_lay="48,32", dnn_act="relu,relu",
                dnn_drop="0.0,0.0", dnn_use_batchnorm="True,True", dnn_use_laynorm="False,False",
                param_quant="8,8", mlp_prune_perc="70,70",
                arch_library="neural_networks", arch_class="MLP", arch_freeze="False",
                arch_seq_model="False", arch_lr="0.08", arch_opt="sgd", opt_momentum="0.0",
                opt_weight_decay="0.0", opt_dampening="0.0", opt_nesterov="False")
    head = dict(MLP_DEF, arch_name="MLP_layers2", dnn_lay="96", dnn_act="softmax",
                dnn_use_batchnorm="False", arch_library="neural_networks", arch_class="MLP",
                arch_freeze="False", arch_seq_model="False", arch_lr="0.0004", arch_opt="rmsprop",
                opt_momentum="0.0", opt_alpha="0.95", opt_eps="1e-8", opt_centered="False",
                opt_weight_decay="0.0")
    mono = dict(head, arch_name="MLP_layers3", dnn_lay="8")
    if variant == "hcgs":
        body.update(mlp_hcgs="True", hcgs_block="16,4", hcgs_sparse="50,50")
        head.update(mlp_hcgs="True", hcgs_block="16,4", hcgs_sparse="25,50")
    if variant == "quant":
        for d in (body, head, mono):
            d.update(mlp_quant="True", mlp_quant_inp="True")
    if variant == "ln":
        body.update(dnn_use_batchnorm="False,True", dnn_use_laynorm="True,True",
                    dnn_use_batchnorm_inp="True", dnn_act="relu,tanh")
    reg = REG_LINES.get(variant)
    if reg:                        # regularised body + mono head, skipped cd head (utils.py:24-60)
        body.update(skip_regularization="False")
        mono.update(skip_regularization="False")
    cfg["architecture1"] = body
    cfg["architecture2"] = head
    cfg["architecture3"] = mono
    tail = ("loss_tmp=sum(loss_cd,loss_mono_w)\n" + reg + "\nloss_final=sum(loss_tmp,%s)\n"
            % reg.split("=")[0]) if reg else "loss_final=sum(loss_cd,loss_mono_w)\n"
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,fmllr)\n"
                             "out_dnn2=compute(MLP_layers2,out_dnn1)\n"
                             "out_dnn3=compute(MLP_layers3,out_dnn1)\n"
                             "loss_mono=cost_nll(out_dnn3,lab_mono)\n"
                             "loss_mono_w=mult_constant(loss_mono,1.0)\n"
                             "loss_cd=cost_nll(out_dnn2,lab_cd)\n" + tail +
                             "err_final=cost_err(out_dnn2,lab_cd)"}
    return cfg


# [model] lines of the regulariser variants (cfg/TIMIT_CGS/TIMIT_LSTM_fmllr_L1.cfg,
# ..._groupLasso.cfg use these forms; lambdas scaled up so the term is visible at this size)
REG_LINES = {"l1": "loss_l1=cost_l1(out_dnn2,0.01)",
             "l2": "loss_l2=cost_l2(out_dnn2,0.05)",
             "gl": "loss_gl=cost_gl(out_dnn2,0.02,3)"}



LIGRU_DEF = dict(ligru_lay="16,16", ligru_drop="0.0,0.0", ligru_use_laynorm_inp="False",
                 ligru_use_batchnorm_inp="False", ligru_use_laynorm="False,False",
                 ligru_use_batchnorm="True,True", ligru_bidir="True", ligru_act="relu,relu",
                 ligru_orthinit="True", use_cuda="False", to_do="train")
LSTM_DEF = dict(lstm_lay="16,16", lstm_drop="0.0,0.0", lstm_use_laynorm_inp="False",
                lstm_use_batchnorm_inp="False", lstm_use_laynorm="False,False",
                lstm_use_batchnorm="True,True", lstm_bidir="False", lstm_act="tanh,tanh",
                lstm_orthinit="True", use_cuda="False", to_do="train", lstm_hcgs="False",
                hcgsx_block="8,2", hcgsh_block="8,2", hcgsx_sparse="50,50", hcgsh_sparse="50,50",
                out_folder=_TMP, lstm_quant="False", param_quant="8,8", lstm_quant_inp="False",
                inp_quant="16", lstm_prune="False", lstm_prune_perc="70,70",
                skip_regularization="True", guided_hcgs="False", apply_guided_hcgs="False",
                if_hsigmoid="True", arch_name="LSTM_layers")




# guided HCGS known answers (make_golden.gen_ghcgs): (shape, block sizes, drop ratios); case 4 has
# exactly tied block means, case 1 selects no block at all (round(2 * 0.1875) = 0)
GHCGS = [((48, 40), [16, 4], [50, 50]), ((64, 64), [32], [81.25]), ((30, 20), [8, 2], [50, 50]),
         ((100, 70), [32, 4], [75, 50]), ((96, 96), [32, 8], [50, 25])]


GRU_DEF = dict(gru_lay="16,16", gru_drop="0.0,0.0", gru_use_laynorm_inp="False",
               gru_use_batchnorm_inp="False", gru_use_laynorm="False,False",
               gru_use_batchnorm="True,True", gru_bidir="True", gru_act="relu,relu",
               gru_orthinit="True", use_cuda="False", to_do="train")
# (tag, options, T, B, F, seed) of the GRU golden cases (tests/golden/gru.npz)
GRU_CASES = [("gru_bidir", GRU_DEF, 7, 3, 20, 31),
             ("gru_uni_nobn", dict(GRU_DEF, gru_bidir="False", gru_use_batchnorm="False,False",
                                   gru_act="tanh,tanh", gru_orthinit="False"), 6, 2, 12, 32)]

MINGRU_DEF = {k.replace("gru_", "minimalgru_"): v for k, v in GRU_DEF.items()}
RNN_DEF = {k.replace("gru_", "rnn_"): v for k, v in GRU_DEF.items()}
# (tag, class, options, T, B, F, seed): minimalGRU / RNN golden cases (tests/golden/gru.npz)
PLAIN_CASES = [("mingru_bidir", "minimalGRU", MINGRU_DEF, 7, 3, 20, 33),
               ("mingru_uni_nobn", "minimalGRU", dict(MINGRU_DEF, minimalgru_bidir="False",
                                                       minimalgru_use_batchnorm="False,False",
                                                       minimalgru_act="tanh,tanh",
                                                       minimalgru_orthinit="False"), 6, 2, 12, 34),
               ("rnn_bidir", "RNN", RNN_DEF, 7, 3, 20, 35),
               ("rnn_uni_nobn", "RNN", dict(RNN_DEF, rnn_bidir="False",
                                            rnn_use_batchnorm="False,False", rnn_act="tanh,relu",
                                            rnn_orthinit="False"), 6, 2, 12, 36)]


# run_nn chunk-lifecycle golden cases (make_golden.gen_run_nn / tests/test_gpu_run_nn_parity.py)
RUN_NN_CASES = ("mlp", "ligru", "lstm_quant")


def run_nn_cfg(d, name, to_do, scp, case, pretrain=None, counts="none"):
    """A chunk cfg in the reference's schema (what utils.create_chunks writes) for the run_nn
    golden case `case`; pretrain: {section: pkl path}."""
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"seed": "2234", "out_folder": d, "use_cuda": "False", "multi_gpu": "False",
                  "to_do": to_do, "out_info": os.path.join(d, name + ".info"),
                  "save_gpumem": "False", "production": "False", "run_nn_script": "run_nn.py"}
    seq = case != "mlp"
    cfg["batches"] = {"batch_size_train": "4" if seq else "16",
                      "batch_size_valid": "4" if seq else "16",
                      "max_seq_length_train": "30", "max_seq_length_valid": "1000"}
    cfg["data_chunk"] = {
        "fea": "fea_name=fmllr\nfea_lst=%s\nfea_opts=\ncw_left=2\ncw_right=2\n" % scp,
        "lab": "lab_name=lab_cd\nlab_folder=%s\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=%s\nlab_opts=ali-to-phones --per-frame=true\n"
               % (scp + ".ali", scp + ".ali")}
    common = dict(arch_library="neural_networks", arch_freeze="False", out_folder=d,
                  arch_pretrain_file="none", use_cuda="False")
    if case == "mlp":
        body = dict(MLP_DEF, **common, arch_name="MLP_layers1", arch_class="MLP",
                    arch_seq_model="False", dnn_lay="64,64", dnn_act="relu,relu",
                    dnn_drop="0.0,0.0", dnn_use_batchnorm="True,True",
                    dnn_use_laynorm="False,False", param_quant="8,8", mlp_prune_perc="70,70",
                    arch_lr="0.08", arch_opt="sgd", opt_momentum="0.5", opt_weight_decay="0.0",
                    opt_dampening="0.0", opt_nesterov="False")
    elif case == "ligru":
        body = dict(LIGRU_DEF, **common, arch_name="RNN_layers", arch_class="liGRU",
                    arch_seq_model="True", ligru_lay="24,24", arch_lr="0.0016", arch_opt="rmsprop",
                    opt_momentum="0.0", opt_alpha="0.95", opt_eps="1e-8", opt_centered="False",
                    opt_weight_decay="0.0")
    else:
        body = dict(LSTM_DEF, **common, arch_name="RNN_layers", arch_class="LSTM",
                    arch_seq_model="True", lstm_lay="24,24", lstm_quant="True",
                    lstm_quant_inp="True", arch_lr="0.0016", arch_opt="rmsprop",
                    opt_momentum="0.0", opt_alpha="0.95", opt_eps="1e-8", opt_centered="False",
                    opt_weight_decay="0.0")
    head = dict(MLP_DEF, **common, arch_name="MLP_layers2", arch_class="MLP",
                arch_seq_model="False", dnn_lay="48", dnn_act="softmax",
                dnn_use_batchnorm="False", arch_lr="0.0004", arch_opt="rmsprop",
                opt_momentum="0.0", opt_alpha="0.95", opt_eps="1e-8", opt_centered="False",
                opt_weight_decay="0.0")
    mono = dict(head, arch_name="MLP_layers3", dnn_lay="8", arch_opt="adam", opt_betas="0.9,0.999",
                opt_eps="1e-8", opt_weight_decay="0.0", opt_amsgrad="False", arch_lr="0.001")
    for sec, a in (("architecture1", body), ("architecture2", head), ("architecture3", mono)):
        cfg[sec] = a
        cfg[sec]["to_do"] = to_do
        if pretrain:
            cfg[sec]["arch_pretrain_file"] = pretrain[sec]
    b = body["arch_name"]
    cfg["model"] = {"model": "out_dnn1=compute(%s,fmllr)\n"
                             "out_dnn2=compute(MLP_layers2,out_dnn1)\n"
                             "out_dnn3=compute(MLP_layers3,out_dnn1)\n"
                             "loss_mono=cost_nll(out_dnn3,lab_mono)\n"
                             "loss_mono_w=mult_constant(loss_mono,1.0)\n"
                             "loss_cd=cost_nll(out_dnn2,lab_cd)\n"
                             "loss_final=sum(loss_cd,loss_mono_w)\n"
                             "err_final=cost_err(out_dnn2,lab_cd)" % b}
    cfg["forward"] = {"forward_out": "out_dnn2", "normalize_posteriors": "True",
                      "normalize_with_counts_from": counts, "save_out_file": "True",
                      "require_decoding": "True"}
    path = os.path.join(d, name + ".cfg")
    with open(path, "w") as f:
        cfg.write(f)
    return path
