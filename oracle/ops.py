"""ORACLE (test infrastructure only): CPU restatement of the hot-path arithmetic.

Each function names the reference file:line it restates (paths under /root/reference/FoodRec).
torch-CPU is used for the float ops because the reference itself is PyTorch (its arithmetic
lives in ATen); numpy/scipy for the integer graph construction.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch


# ----------------------------------------------------------------------------- row gathers
def embedding_bwd_f64(idx, G, num_rows: int, padding_idx=None) -> np.ndarray:
    """Weight gradient of a row gather ``W[idx]`` / ``nn.Embedding(idx)`` in float64.

    Restates the autograd of ``ingr_all_embeddings[ingredients]`` (cikm_model.py:230; index
    backward = index_put_ accumulate) and of ``self.ingre_embedding(...)`` with
    ``padding_idx=self.n_ingredients`` (cikm_model.py:67-68, 270-271; embedding backward leaves the
    padding row's gradient zero): dW[r] = sum_{i : idx[i] == r, r != padding_idx} G[i].
    """
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    G = np.asarray(G, dtype=np.float64)
    G = G.reshape(idx.shape[0], G.shape[-1])
    keep = idx != (-1 if padding_idx is None else int(padding_idx))
    out = np.zeros((num_rows, G.shape[1]), np.float64)
    np.add.at(out, idx[keep], G[keep])
    return out


# ----------------------------------------------------------------------------- adjacency
def norm_adj_coo(n_nodes: int, rows, cols):
    """D^-1/2 A D^-1/2 of the symmetrised binary graph.

    Restates get_norm_adj_mat (models/lightgcn.py:76-120, cikm_model.py:136-180) and
    get_norm_adj_recipe_ing / _infor (cikm_model.py:112-134, pricai_modelx.py:109-131):
    dok insert of (r,c) and (c,r) with value 1 (duplicates collapse), deg = (A>0).sum(1) + 1e-7,
    diag = deg^-0.5 (float64), L = D*A*D, coo order, values cast to float32.
    Returns (row int64, col int64, val float32) in row-major sorted order.
    """
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    A = sp.coo_matrix((np.ones(2 * len(rows), np.float32),
                       (np.concatenate([rows, cols]), np.concatenate([cols, rows]))),
                      shape=(n_nodes, n_nodes)).tocsr()
    A.data[:] = 1.0  # binary: the dok dict keeps one entry per (r, c)
    deg = np.asarray((A > 0).sum(axis=1)).ravel() + 1e-7
    D = sp.diags(np.power(deg, -0.5))
    L = sp.coo_matrix(D * A * D)
    order = np.lexsort((L.col, L.row))
    return L.row[order].astype(np.int64), L.col[order].astype(np.int64), L.data[order].astype(np.float32)


def coo_to_torch(n_nodes, row, col, val) -> torch.Tensor:
    i = torch.from_numpy(np.stack([row, col]))
    return torch.sparse_coo_tensor(i, torch.from_numpy(val), (n_nodes, n_nodes)).coalesce()


# ----------------------------------------------------------------------------- propagation
def propagate_mean(adj: torch.Tensor, ego: torch.Tensor, n_layers: int) -> torch.Tensor:
    """LightGCN layer stack + mean (models/lightgcn.py:134-144, cikm_model.py:182-208)."""
    out = [ego]
    x = ego
    for _ in range(n_layers):
        x = torch.sparse.mm(adj, x)
        out.append(x)
    return torch.stack(out, dim=1).mean(dim=1)


def spmm_f64(row, col, val, n_rows, X: np.ndarray) -> np.ndarray:
    A = sp.csr_matrix((val.astype(np.float64), (row, col)), shape=(n_rows, X.shape[0]))
    return A @ X.astype(np.float64)


# ----------------------------------------------------------------------------- losses
def bpr_loss(pos_score: torch.Tensor, neg_score: torch.Tensor, gamma: float = 1e-10) -> torch.Tensor:
    """common/loss.py:29-34."""
    return -torch.log(gamma + torch.sigmoid(pos_score - neg_score)).mean()


def emb_loss(*embeddings: torch.Tensor) -> torch.Tensor:
    """common/loss.py:45-50: sum of Frobenius norms / rows of the LAST argument, shape [1]."""
    total = torch.zeros(1, dtype=embeddings[-1].dtype)
    for e in embeddings:
        total = total + torch.norm(e, p=2)
    return total / embeddings[-1].shape[0]


def correlation_distance(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """models/pricai_modelx.py:409-437 (distance correlation of two [n,d] views), shape [1]."""
    zero = torch.zeros(1, dtype=x.dtype)

    def centred(X):
        r = (X * X).sum(1, keepdim=True)
        q = r - 2 * X @ X.t() + r.t()
        D = torch.sqrt(torch.maximum(q, zero) + 1e-8)
        return D - D.mean(0, keepdim=True) - D.mean(1, keepdim=True) + D.mean()

    def dcov(D1, D2):
        n = D1.shape[0]
        s = (D1 * D2).sum() / (torch.ones(1, dtype=x.dtype) * n * n)
        return torch.sqrt(torch.maximum(s, zero) + 1e-8)

    A, B = centred(x), centred(y)
    c12, c11, c22 = dcov(A, B), dcov(A, A), dcov(B, B)
    return c12 / torch.sqrt(torch.maximum(c11 * c22, zero) + 1e-10)


def cl_loss(hidden: torch.Tensor, temperature: float = 0.5) -> torch.Tensor:
    """models/pricai_modelx.py:354-378 (InfoNCE over two halves, hidden_norm=True)."""
    b = hidden.shape[0] // 2
    h = torch.nn.functional.normalize(hidden, p=2, dim=-1)
    h1, h2 = h[:b], h[b:2 * b]
    labels = torch.arange(b)
    mask = torch.eye(b, dtype=hidden.dtype) * 1e9
    aa = h1 @ h1.t() / temperature - mask
    bb = h2 @ h2.t() / temperature - mask
    ab = h1 @ h2.t() / temperature
    ba = h2 @ h1.t() / temperature
    la = torch.nn.functional.cross_entropy(torch.cat([ab, aa], 1), labels)
    lb = torch.nn.functional.cross_entropy(torch.cat([ba, bb], 1), labels)
    return (la + lb) / b


def bpr_step_reference(U_all, I_all, U_ego, I_ego, user, pos, neg, reg_weight, gamma=1e-10):
    """Gather/dot/BPR + weighted EmbLoss exactly as models/lightgcn.py:158-177 composes them."""
    u, p, n = U_all[user], I_all[pos], I_all[neg]
    mf = bpr_loss((u * p).sum(1), (u * n).sum(1), gamma)
    reg = reg_weight * emb_loss(U_ego[user], I_ego[pos], I_ego[neg])
    return mf, reg


# ----------------------------------------------------------------------------- full-sort top-k
def full_sort_topk(U: np.ndarray, I: np.ndarray, k: int, exclude=None, held_out=None):
    """Full-sort ranking of every item for each user row of U.

    Restates Trainer.evaluate (common/trainer.py:476-503): scores = full_sort_predict (the dense
    user @ item.T of common/abstract_recommender.py:39-50), torch.topk(scores, max(topk)); with
    the MMRec history mask (scores of ``exclude[u]`` items set to -inf before the top-k) when
    ``exclude`` is given; hits = ``i in pos_items`` of TopKEvaluator.evaluate
    (utils/topk_evaluator.py:104-107) against ``held_out[u]``.  Scores in float64 on the given
    values; ties ordered by item id (a stable descending sort: torch.topk leaves tie order
    unspecified).  Returns (scores [n,k] f64, items [n,k] int64, hits [n,k] bool or None).
    """
    S = np.asarray(U, np.float64) @ np.asarray(I, np.float64).T
    n = S.shape[0]
    if exclude is not None:
        for u in range(n):
            ex = np.asarray(list(exclude[u]), np.int64)
            if ex.size:
                S[u, ex] = -np.inf
    order = np.argsort(-S, axis=1, kind="stable")[:, :k]
    scores = np.take_along_axis(S, order, 1)
    hits = None
    if held_out is not None:
        hits = np.array([[i in set(held_out[u]) for i in order[u]] for u in range(n)], dtype=bool)
    return scores, order.astype(np.int64), hits


def bf16_round(x) -> np.ndarray:
    """float32 values rounded to bfloat16 (round to nearest even), returned as float32."""
    return torch.as_tensor(np.asarray(x, np.float32)).to(torch.bfloat16).float().numpy()


# ----------------------------------------------------------------------------- encoder layer
def _mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def encoder_keep_masks(seed: int, counter: int, n_seq: int, L: int, drop, heads: int = 2, d: int = 64,
                       ff: int = 256):
    """The fused encoder's dropout keep-masks (fr_encoder.hip: site_keys / keep), restated in numpy.
    key = mix64(seed ^ mix64(counter + C)); site key k_s = hi32(mix64(key + s + 1)); elements 2m and
    2m+1 of site s share h = lowbias32(m * 0x9E3779B1 + k_s) (uint32 arithmetic), and element e is
    kept iff the (e & 1) 16-bit half of h (low half for even e) is >= floor(p * 2^16).
    Sites: 0 attention probs [n_seq, heads, L, L], 1 out-proj [n_seq, L, d], 2 FF activation
    [n_seq, L, ff], 3 FF out [n_seq, L, d] (element index = row-major position).  Returns 4 float64
    arrays of 0/1."""
    shapes = [(n_seq, heads, L, L), (n_seq, L, d), (n_seq, L, ff), (n_seq, L, d)]
    out = []
    u32 = np.uint32
    with np.errstate(over="ignore"):
        key = _mix64(np.array([seed], np.uint64) ^ _mix64(np.array([counter], np.uint64)
                                                          + np.uint64(0x632BE59BD9B4E019)))
        for site, (shape, p) in enumerate(zip(shapes, drop)):
            if p == 0:
                out.append(np.ones(shape))
                continue
            thr = min(int(float(np.float32(p)) * 65536.0), 65535)
            ks = (_mix64(key + np.uint64(site + 1)) >> np.uint64(32)).astype(u32)
            e = np.arange(int(np.prod(shape)), dtype=np.uint64).astype(u32)
            x = (e >> u32(1)) * u32(0x9E3779B1) + ks
            x ^= x >> u32(16)
            x *= u32(0x7FEB352D)
            x ^= x >> u32(15)
            x *= u32(0x846CA68B)
            x ^= x >> u32(16)
            half = np.where(e & u32(1), x >> u32(16), x & u32(0xFFFF))
            out.append((half >= u32(thr)).astype(np.float64).reshape(shape))
    return out


def encoder_layer_f64(x, mask, params, masks, drop, eps=(1e-5, 1e-5), gelu=True, heads: int = 2):
    """nn.TransformerEncoderLayer's post-norm training forward (torch/nn/modules/transformer.py,
    built at cikm_model.py:33-35) in float64 torch-CPU, batch-first x [n_seq, L, d], additive key
    mask [n_seq, L] (or None), with explicit dropout keep-masks (encoder_keep_masks) scaled by
    1/(1-p).  Differentiable: used for the gradient references."""
    w_in, b_in, w_o, b_o, g1, be1, w1, b1, w2, b2, g2, be2 = params
    NS, L, d = x.shape
    hd = d // heads
    ma, m1, mf, m2 = (torch.as_tensor(m, dtype=torch.float64) / (1.0 - p) for m, p in zip(masks, drop))
    qkv = x @ w_in.t() + b_in
    q, k, v = (t.reshape(NS, L, heads, hd).transpose(1, 2) for t in qkv.split(d, dim=-1))
    s = q @ k.transpose(-1, -2) * hd ** -0.5
    if mask is not None:
        s = s + mask.view(NS, 1, 1, L)
    pa = torch.softmax(s, dim=-1) * ma
    ctx = (pa @ v).transpose(1, 2).reshape(NS, L, d)
    y1 = x + (ctx @ w_o.t() + b_o) * m1
    x1 = torch.nn.functional.layer_norm(y1, (d,), g1, be1, eps[0])
    pre = x1 @ w1.t() + b1
    f = (torch.nn.functional.gelu(pre) if gelu else torch.relu(pre)) * mf
    y2 = x1 + (f @ w2.t() + b2) * m2
    return torch.nn.functional.layer_norm(y2, (d,), g2, be2, eps[1])


# ----------------------------------------------------------------------------- modal fusion
def target_attention_f64(q_in, kv_in, ln_w, ln_b, eps, num_head=2, seq_ids=None, padding_idx=None):
    """target_attention_layer.forward with atten_mode='ln', linear_projection=False
    (models/cikm_model.py:325-369), float64 torch-CPU: head split by chunk/cat, the module's
    LayerNorm on the q and k heads, scores / sqrt(d/h), padded keys -> keep*s + pad*(-2**32+1),
    softmax, @ v, heads concatenated back."""
    Q_ = torch.cat(torch.chunk(q_in, num_head, dim=2), dim=0)
    K_ = torch.cat(torch.chunk(kv_in, num_head, dim=2), dim=0)
    V_ = torch.cat(torch.chunk(kv_in, num_head, dim=2), dim=0)
    d = Q_.shape[-1]
    Q_ = torch.nn.functional.layer_norm(Q_, (d,), ln_w, ln_b, eps)
    K_ = torch.nn.functional.layer_norm(K_, (d,), ln_w, ln_b, eps)
    out = torch.matmul(Q_, K_.permute(0, 2, 1)) * (K_.shape[-1] ** (-0.5))
    if seq_ids is not None:
        lq, lk = q_in.shape[1], kv_in.shape[1]
        key_masks = ((seq_ids == padding_idx).double() * (-2 ** 32 + 1)).view(-1, 1, lk).repeat(num_head, lq, 1)
        out = (seq_ids != padding_idx).double().view(-1, 1, lk).repeat(num_head, lq, 1) * out + key_masks
    out = torch.softmax(out, dim=-1)
    out = torch.matmul(out, V_)
    return torch.cat(torch.chunk(out, num_head, dim=0), dim=2)


def modal_fusion_f64(enc, query, ids, num, pad_id, ln_a, ln_b, eps=1e-12):
    """cikm_model.py:245-249 in float64: item_health = mm_target_atten(query, enc, ids),
    item_mm = ingre_target_atten(enc, query); returns (F.normalize(item_mm).sum(1) / num,
    F.normalize(item_health).mean(1))."""
    item_health = target_attention_f64(query, enc, ln_a[0], ln_a[1], eps, seq_ids=ids, padding_idx=pad_id)
    item_mm = target_attention_f64(enc, query, ln_b[0], ln_b[1], eps)
    know = torch.nn.functional.normalize(item_mm).sum(1) / num.unsqueeze(1)
    hin = torch.nn.functional.normalize(item_health).mean(dim=1)
    return know, hin


def health_kd_f64(hin, know, rows, labels, w1, b1, w2, b2, kd_threshold, w_health, w_kd):
    """HealthRec's loss head in float64 (cikm_model.py:249-264 and norm_loss :304-308):
    (w_health * sum BCELoss(sigmoid(Linear2(relu(Linear1(hin)))), labels),
     w_kd * max(0, 1 - cosine_similarity(know, rows, dim=-1).mean() - kd_threshold)).
    Inputs are float64 torch tensors (requires_grad as the test needs)."""
    F = torch.nn.functional
    pred = torch.sigmoid(F.linear(torch.relu(F.linear(hin, w1, b1)), w2, b2))
    health = torch.sum(torch.nn.BCELoss(reduction="none")(pred, labels))
    kd = 1 - F.cosine_similarity(know, rows, dim=-1).mean()
    kd = torch.max(torch.zeros((), dtype=kd.dtype), kd - kd_threshold)
    return w_health * health, w_kd * kd


def gcn_conv_f64(x, edge_index, weight, bias, edge_weight=None, improved=False):
    """PyG GCNConv (documented semantics; PyG is not installed, parity unpinned) in float64 with
    explicit per-edge loops: add_remaining_self_loops (fill 1 / 2 if improved; an existing loop
    keeps its weight), deg over targets, w = deg^-1/2[src] w deg^-1/2[dst], out[dst] += w (x W^T)[src],
    + bias.  x [N, in], edge_index [2, E] (src, dst), weight [out, in]."""
    x = np.asarray(x, np.float64)
    ei = np.asarray(edge_index, np.int64)
    N = x.shape[0]
    w_in = np.ones(ei.shape[1]) if edge_weight is None else np.asarray(edge_weight, np.float64)
    loop_w = np.full(N, 2.0 if improved else 1.0)
    edges = []
    for e in range(ei.shape[1]):
        s, d = int(ei[0, e]), int(ei[1, e])
        if s == d:
            loop_w[s] = w_in[e]
        else:
            edges.append((s, d, w_in[e]))
    edges += [(i, i, loop_w[i]) for i in range(N)]
    deg = np.zeros(N)
    for s, d, w in edges:
        deg[d] += w
    dinv = np.where(deg > 0, deg ** -0.5, 0.0)
    h = x @ np.asarray(weight, np.float64).T
    out = np.zeros((N, h.shape[1]))
    for s, d, w in edges:
        out[d] += dinv[s] * w * dinv[d] * h[s]
    return out + (0.0 if bias is None else np.asarray(bias, np.float64))
