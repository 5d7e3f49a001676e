"""Euclidean RE-GCN (mirror of src/rrgcn.py, src/model.py, src/decoder.py) on HIP.

`RecurrentRGCN.forward(g_list, static_graph, use_cuda)` keeps the reference signature and
5-tuple return (src/rrgcn.py:142-180).  Message passing and the relation-context mean
run on HIP; the relation GRU, the time gate and the ConvTransE/R decoders stay on torch
(host GEMMs).  With autograd on (training), forward runs
training.euclid_model_forward (HIP aggregation forward + backward); get_loss mirrors
src/rrgcn.py:196-248 without the static graph.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.parameter import Parameter

from . import autograd as _ag
from .hyperbolic_model import relation_gru_step
from .layers import UnionRGCNLayer


class BaseRGCN(nn.Module):
    """src/model.py:4-71."""

    def __init__(self, num_nodes, h_dim, out_dim, num_rels, num_bases=-1, num_basis=-1, num_hidden_layers=1,
                 dropout=0, self_loop=False, skip_connect=False, encoder_name="", opn="sub", rel_emb=None,
                 use_cuda=False, analysis=False):
        super().__init__()
        self.num_nodes, self.h_dim, self.out_dim, self.num_rels = num_nodes, h_dim, out_dim, num_rels
        self.num_bases, self.num_basis, self.num_hidden_layers = num_bases, num_basis, num_hidden_layers
        self.dropout, self.skip_connect, self.self_loop = dropout, skip_connect, self_loop
        self.encoder_name, self.use_cuda, self.run_analysis = encoder_name, use_cuda, analysis
        self.rel_emb, self.opn = rel_emb, opn
        self.layers = nn.ModuleList([self.build_hidden_layer(i) for i in range(num_hidden_layers)])
        self.features = None


class RGCNCell(BaseRGCN):
    """src/rrgcn.py:14-54 (encoder 'uvrgcn')."""

    def build_hidden_layer(self, idx):
        if self.encoder_name != "uvrgcn":
            raise NotImplementedError
        sc = (idx != 0) if self.skip_connect else False
        if self.run_analysis:  # src/rrgcn.py:19-20
            print("activate function: {}".format(F.rrelu))
        return UnionRGCNLayer(self.h_dim, self.h_dim, self.num_rels, self.num_bases, activation=F.rrelu,
                              dropout=self.dropout, self_loop=self.self_loop, skip_connect=sc, rel_emb=self.rel_emb)

    def forward(self, g, init_ent_emb, init_rel_emb):
        g.ndata["h"] = init_ent_emb
        for i, layer in enumerate(self.layers):
            layer(g, [], init_rel_emb[i])
        return g.ndata.pop("h")


class ConvTransE(nn.Module):
    """src/decoder.py:55-100."""

    def __init__(self, num_entities, embedding_dim, input_dropout=0, hidden_dropout=0, feature_map_dropout=0,
                 channels=50, kernel_size=3, use_bias=True):
        super().__init__()
        self.inp_drop = nn.Dropout(input_dropout)
        self.hidden_drop = nn.Dropout(hidden_dropout)
        self.feature_map_drop = nn.Dropout(feature_map_dropout)
        self.loss = nn.BCELoss()
        self.conv1 = nn.Conv1d(2, channels, kernel_size, stride=1, padding=int(math.floor(kernel_size / 2)))
        self.bn0 = nn.BatchNorm1d(2)
        self.bn1 = nn.BatchNorm1d(channels)
        self.bn2 = nn.BatchNorm1d(embedding_dim)
        self.register_parameter("b", Parameter(torch.zeros(num_entities)))
        self.fc = nn.Linear(embedding_dim * channels, embedding_dim)
        self.bn3 = nn.BatchNorm1d(embedding_dim)
        self.bn_init = nn.BatchNorm1d(embedding_dim)

    def forward(self, embedding, emb_rel, triplets, nodes_id=None, mode="train", negative_rate=0,
                partial_embeding=None):
        e_all = torch.tanh(embedding)
        B = len(triplets)
        x = torch.cat([e_all[triplets[:, 0]].unsqueeze(1), emb_rel[triplets[:, 1]].unsqueeze(1)], 1)
        x = self.feature_map_drop(F.relu(_ag.batch_norm(self.bn1, self.conv1(self.inp_drop(_ag.batch_norm(self.bn0, x))))))
        x = self.hidden_drop(_ag.linear(self.fc, x.view(B, -1)))
        if B > 1:
            x = _ag.batch_norm(self.bn2, x)
        x = F.relu(x)
        return torch.mm(x, (e_all if partial_embeding is None else partial_embeding).transpose(1, 0))


class ConvTransR(nn.Module):
    """src/decoder.py:10-52."""

    def __init__(self, num_relations, embedding_dim, input_dropout=0, hidden_dropout=0, feature_map_dropout=0,
                 channels=50, kernel_size=3, use_bias=True):
        super().__init__()
        self.inp_drop = nn.Dropout(input_dropout)
        self.hidden_drop = nn.Dropout(hidden_dropout)
        self.feature_map_drop = nn.Dropout(feature_map_dropout)
        self.loss = nn.BCELoss()
        self.conv1 = nn.Conv1d(2, channels, kernel_size, stride=1, padding=int(math.floor(kernel_size / 2)))
        self.bn0 = nn.BatchNorm1d(2)
        self.bn1 = nn.BatchNorm1d(channels)
        self.bn2 = nn.BatchNorm1d(embedding_dim)
        self.register_parameter("b", Parameter(torch.zeros(num_relations * 2)))
        self.fc = nn.Linear(embedding_dim * channels, embedding_dim)
        self.bn3 = nn.BatchNorm1d(embedding_dim)
        self.bn_init = nn.BatchNorm1d(embedding_dim)

    def forward(self, embedding, emb_rel, triplets, nodes_id=None, mode="train", negative_rate=0):
        e_all = torch.tanh(embedding)
        B = len(triplets)
        x = torch.cat([e_all[triplets[:, 0]].unsqueeze(1), e_all[triplets[:, 2]].unsqueeze(1)], 1)
        x = self.feature_map_drop(F.relu(_ag.batch_norm(self.bn1, self.conv1(self.inp_drop(_ag.batch_norm(self.bn0, x))))))
        x = _ag.batch_norm(self.bn2, self.hidden_drop(_ag.linear(self.fc, x.view(B, -1))))
        return torch.mm(F.relu(x), emb_rel.transpose(1, 0))


class RecurrentRGCN(nn.Module):
    """src/rrgcn.py:58-248."""

    def __init__(self, decoder_name, encoder_name, num_ents, num_rels, num_static_rels, num_words, h_dim, opn,
                 sequence_len, num_bases=-1, num_basis=-1, num_hidden_layers=1, dropout=0, self_loop=False,
                 skip_connect=False, layer_norm=False, input_dropout=0, hidden_dropout=0, feat_dropout=0,
                 aggregation="cat", weight=1, discount=0, angle=0, use_static=False, entity_prediction=False,
                 relation_prediction=False, use_cuda=False, gpu=0, analysis=False):
        super().__init__()
        if use_static:
            raise NotImplementedError("static graph is outside this build's scope (SURVEY.md §2 row 1)")
        self.decoder_name, self.encoder_name, self.num_rels, self.num_ents = decoder_name, encoder_name, num_rels, \
            num_ents
        self.opn, self.num_words, self.num_static_rels, self.sequence_len = opn, num_words, num_static_rels, \
            sequence_len
        self.h_dim, self.layer_norm, self.h, self.run_analysis = h_dim, layer_norm, None, analysis
        self.aggregation, self.relation_evolve, self.weight, self.discount = aggregation, False, weight, discount
        self.use_static, self.angle = use_static, angle
        self.relation_prediction, self.entity_prediction, self.gpu = relation_prediction, entity_prediction, gpu
        self.w1 = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_normal_(self.w1)
        self.w2 = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_normal_(self.w2)
        self.emb_rel = nn.Parameter(torch.Tensor(num_rels * 2, h_dim))
        nn.init.xavier_normal_(self.emb_rel)
        self.dynamic_emb = nn.Parameter(torch.Tensor(num_ents, h_dim))
        nn.init.normal_(self.dynamic_emb)
        self.loss_r = nn.CrossEntropyLoss()
        self.loss_e = nn.CrossEntropyLoss()
        self.rgcn = RGCNCell(num_ents, h_dim, h_dim, num_rels * 2, num_bases, num_basis, num_hidden_layers, dropout,
                             self_loop, skip_connect, encoder_name, opn, self.emb_rel, use_cuda, analysis)
        self.time_gate_weight = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_uniform_(self.time_gate_weight, gain=nn.init.calculate_gain("relu"))
        self.time_gate_bias = nn.Parameter(torch.Tensor(h_dim))
        nn.init.zeros_(self.time_gate_bias)
        self.relation_cell_1 = nn.GRUCell(h_dim * 2, h_dim)
        if decoder_name != "convtranse":
            raise NotImplementedError
        self.decoder_ob = ConvTransE(num_ents, h_dim, input_dropout, hidden_dropout, feat_dropout)
        self.rdecoder = ConvTransR(num_rels, h_dim, input_dropout, hidden_dropout, feat_dropout)
        from .weights import invalidate
        self.register_load_state_dict_post_hook(lambda module, _keys: invalidate(module))

    def forward(self, g_list, static_graph, use_cuda):
        """src/rrgcn.py:142-180."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .training import euclid_model_forward
            out = euclid_model_forward(self, g_list)
            self.h, self.h_0 = out[0][-1], out[2]
            return out
        dev = self.dynamic_emb.device
        self.h = F.normalize(self.dynamic_emb) if self.layer_norm else self.dynamic_emb[:, :]
        self.h = self.h.contiguous()
        history_embs = []
        R2 = self.num_rels * 2
        for i, g in enumerate(g_list):
            g = g.to(dev)
            self.h_0 = relation_gru_step(self.relation_cell_1, self.emb_rel, self.h, g,
                                         self.emb_rel if i == 0 else self.h_0)
            self.h_0 = F.normalize(self.h_0) if self.layer_norm else self.h_0
            current_h = self.rgcn.forward(g, self.h, [self.h_0, self.h_0])
            current_h = F.normalize(current_h) if self.layer_norm else current_h
            time_weight = torch.sigmoid(torch.mm(self.h, self.time_gate_weight) + self.time_gate_bias)
            self.h = (time_weight * current_h + (1 - time_weight) * self.h).contiguous()
            history_embs.append(self.h)
        return history_embs, None, self.h_0, [], []

    def predict(self, test_graph, num_rels, static_graph, test_triplets, use_cuda):
        """src/rrgcn.py:183-194."""
        with torch.no_grad():
            inv = test_triplets.flip(1)
            inv[:, 1] = inv[:, 1] + num_rels
            all_triples = torch.cat((test_triplets, inv))
            evolve_embs, _, r_emb, _, _ = self.forward(test_graph, static_graph, use_cuda)
            embedding = F.normalize(evolve_embs[-1]) if self.layer_norm else evolve_embs[-1]
            at = all_triples.to(embedding.device)
            return all_triples, self.decoder_ob.forward(embedding, r_emb, at, mode="test"), \
                self.rdecoder.forward(embedding, r_emb, at, mode="test")

    def get_loss(self, glist, triples, static_graph, use_cuda):
        """src/rrgcn.py:196-248 (no static graph): entity / relation cross entropy of the
        ConvTransE / ConvTransR scores over the triples and their inverses."""
        dev = self.dynamic_emb.device
        loss_ent = torch.zeros(1, device=dev)
        loss_rel = torch.zeros(1, device=dev)
        loss_static = torch.zeros(1, device=dev)
        inv = triples[:, [2, 1, 0]].clone()
        inv[:, 1] = inv[:, 1] + self.num_rels
        all_triples = torch.cat([triples, inv]).to(dev)
        evolve_embs, _, r_emb, _, _ = self.forward(glist, static_graph, use_cuda)
        pre_emb = F.normalize(evolve_embs[-1]) if self.layer_norm else evolve_embs[-1]
        if self.entity_prediction:
            scores_ob = self.decoder_ob.forward(pre_emb, r_emb, all_triples).view(-1, self.num_ents)
            loss_ent = loss_ent + self.loss_e(scores_ob, all_triples[:, 2])
        if self.relation_prediction:
            score_rel = self.rdecoder.forward(pre_emb, r_emb, all_triples, mode="train").view(-1, 2 * self.num_rels)
            loss_rel = loss_rel + self.loss_r(score_rel, all_triples[:, 1])
        return loss_ent, loss_rel, loss_static
