"""Shared helpers: replay a golden case through an aggregation engine and compare bit-for-bit.

An *engine* is an object with
    weighted_sum(xs, mode, coef=None, divisor=1.0) -> tensor       (xs: list of same-shape tensors)
    mix(xs, row_ptr, cols, vals, post_scale=None) -> (outs, outs2)
Both the C oracle (oracle.orc) and the HIP product (fedml_amd) are driven through the same
replay, so a case means the same thing for both.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from golden_io import client_dicts, expected_dicts

MUL_W, MUL_N_DIV_N, SUM = 0, 1, 2


def bits_equal(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Bitwise equality; NaN matches NaN (NaN payloads differ between torch CPU paths)."""
    a, b = a.detach().cpu(), b.detach().cpu()
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if not a.is_floating_point():
        return torch.equal(a, b)
    ia = {torch.float32: torch.int32, torch.float64: torch.int64,
          torch.bfloat16: torch.int16, torch.float16: torch.int16}[a.dtype]
    nan = torch.isnan(a) & torch.isnan(b)
    return bool(torch.all((a.view(ia) == b.view(ia)) | nan))


def assert_dict_bits(got: OrderedDict, exp: OrderedDict, what: str = ""):
    assert list(got.keys()) == list(exp.keys()), (what, list(got.keys()), list(exp.keys()))
    for k in exp:
        g, e = got[k], exp[k]
        assert g.dtype == e.dtype, (what, k, g.dtype, e.dtype)
        assert tuple(g.shape) == tuple(e.shape), (what, k, g.shape, e.shape)
        if not bits_equal(g.reshape(-1), e.reshape(-1)):
            gd, ed = g.double().reshape(-1), e.double().reshape(-1)
            bad = torch.nonzero(~((gd == ed) | (torch.isnan(gd) & torch.isnan(ed)))).reshape(-1)
            i = int(bad[0]) if bad.numel() else -1
            raise AssertionError(f"{what} key={k}: {bad.numel()} mismatches, first at {i}: "
                                 f"got {gd[i].item()!r} expected {ed[i].item()!r}")


def per_key(engine, dicts, mode, coef=None, divisor=1.0):
    keys = list(dicts[0].keys())
    out = OrderedDict()
    for k in keys:
        xs = [d[k] for d in dicts]
        shape = xs[0].shape
        r = engine.weighted_sum([x.reshape(-1) for x in xs], mode, coef, divisor)
        out[k] = r.reshape(shape)
    return out


def per_key_mix(engine, dicts, row_ptr, cols, vals, post_scale=None):
    keys = list(dicts[0].keys())
    rows = len(row_ptr) - 1
    outs = [OrderedDict() for _ in range(rows)]
    outs2 = [OrderedDict() for _ in range(rows)] if post_scale is not None else None
    for k in keys:
        shape = dicts[0][k].shape
        o, o2 = engine.mix([d[k].reshape(-1) for d in dicts], row_ptr, cols, vals, post_scale)
        for r in range(rows):
            outs[r][k] = o[r].reshape(shape)
            if outs2 is not None:
                outs2[r][k] = o2[r].reshape(shape)
    return outs, outs2


def dense_csr(W):
    n = W.shape[0]
    row_ptr = [i * n for i in range(n + 1)]
    cols = [j for _ in range(n) for j in range(n)]
    vals = [float(W[i, j]) for i in range(n) for j in range(n)]
    return row_ptr, cols, vals


def dsgd_csr(W):
    """Row i = [self, in-neighbours j ascending] with weights [W_ii, W_ji] (client_dsgd.py:92-116)."""
    n = W.shape[0]
    row_ptr, cols, vals = [0], [], []
    for i in range(n):
        cols.append(i)
        vals.append(float(W[i, i]))
        for j in range(n):
            if j != i and W[j, i] != 0:
                cols.append(j)
                vals.append(float(W[j, i]))
        row_ptr.append(len(cols))
    return row_ptr, cols, vals


def replay(engine, meta, arrays):
    """Return the list of output dicts the reference produced for this case, via `engine`."""
    kind = meta["kind"]
    clients = client_dicts(meta, arrays)
    n = meta.get("n")
    if kind in ("agg", "sp_aggregate"):
        opt = meta.get("optimizer", "FedAvg")
        N = sum(n)
        if opt in ("FedAvg", "FedProx"):
            return [per_key(engine, clients, MUL_W, [v / N for v in n])]
        if opt in ("FedAvg_seq", "FedDyn"):
            return [per_key(engine, clients, SUM)]
        cs = []
        for i in range(meta["num_clients"]):
            d = OrderedDict()
            for key in meta["keys"]:
                d[key] = torch.from_numpy(arrays[f"c{i}__{key}"].copy())
            cs.append(d)
        if opt == "SCAFFOLD":
            K = len(clients)
            if K == 1:
                wout = per_key(engine, clients[:1], MUL_W, [n[0] / N])
            else:
                wout = per_key(engine, clients[-1:], SUM)
            cout = per_key(engine, cs[-1:], MUL_W, [1 / meta["client_num_in_total"]])
            return [wout, cout]
        if opt == "Mime":
            w = [v / N for v in n]
            return [per_key(engine, clients, MUL_W, w), per_key(engine, cs, MUL_W, w)]
        raise ValueError(opt)
    if kind == "mpi_fedavg":
        return [per_key(engine, clients, MUL_N_DIV_N, n, sum(n))]
    if kind == "fedavg_seq":
        N = sum(n)
        partials = [per_key(engine, [clients[i] for i in wk], MUL_W, [n[i] / N for i in wk])
                    for wk in meta["schedule"]]
        return [per_key(engine, partials, SUM)]
    if kind == "hier_sp":
        groups = meta["groups"]
        gw, gn = [], []
        for grp in groups:
            Ng = sum(n[i] for i in grp)
            gw.append(per_key(engine, [clients[i] for i in grp], MUL_W, [n[i] / Ng for i in grp]))
            gn.append(Ng)
        Nt = sum(gn)
        return [per_key(engine, gw, MUL_W, [v / Nt for v in gn])]
    if kind == "hier_cloud":
        E, R, ne = meta["edges"], meta["group_comm_round"], meta["edge_counts"]
        avg = None
        for r in range(R):
            ml = [clients[e * R + r] for e in range(E)]
            cnt = [ne[e][r] for e in range(E)]
            avg = per_key(engine, ml, MUL_N_DIV_N, cnt, sum(cnt))
        ml = [avg] + [clients[e * R + R - 1] for e in range(1, E)]
        cnt = [ne[e][R - 1] for e in range(E)]
        return [per_key(engine, ml, MUL_N_DIV_N, cnt, sum(cnt))]
    if kind == "mix_rows":
        W = arrays["W"]
        outs, _ = per_key_mix(engine, clients, *dense_csr(W))
        return outs
    if kind == "hier_mix":
        E, R = meta["edges"], meta["group_comm_round"]
        W = arrays["W"]
        outs = avg = None
        for r in range(R):
            ml = [clients[e * R + r] for e in range(E)]
            outs, _ = per_key_mix(engine, ml, *dense_csr(W))
            avg = per_key(engine, outs, MUL_N_DIV_N, [1] * E, E)
        return [avg] + outs[1:]
    if kind == "dsgd":
        outs, _ = per_key_mix(engine, clients, *dsgd_csr(arrays["W"]))
        return outs
    if kind == "pushsum":
        scale = [1.0 / o for o in meta["omegas_out"]]
        _, z = per_key_mix(engine, clients, *dsgd_csr(arrays["W"]), post_scale=scale)
        return z
    raise ValueError(kind)


def check_case(engine, meta, arrays, what=""):
    got = replay(engine, meta, arrays)
    exp = expected_dicts(meta, arrays)
    assert len(got) == len(exp), (what, len(got), len(exp))
    for j, (g, e) in enumerate(zip(got, exp)):
        assert_dict_bits(g, e, f"{what}{meta['name']}[{j}]")


def fedopt_replay(meta, arrays, weighted_sum, sgd_apply, to_dev=lambda t: t):
    """Replay a FedOpt fixture: per round FedAvg (weighted_sum), then the SGD server step on the
    parameters (sgd_apply, in place) and the averaged buffers cast into their dtype.  Returns the
    list of per-round global state_dicts (CPU)."""
    from golden_io import np_to_tensor
    keys, dtypes, params = meta["keys"], meta["dtypes"], set(meta["params"])
    state = OrderedDict((k, to_dev(np_to_tensor(arrays[f"init__{k}"], dt))) for k, dt in zip(keys, dtypes))
    bufs = {}
    outs = []
    for r, rd in enumerate(meta["rounds"]):
        n = rd["n"]
        N = sum(n)
        W = len(n)
        new = OrderedDict()
        for k, dt in zip(keys, dtypes):
            xs = [to_dev(np_to_tensor(arrays[f"r{r}_x{i}__{k}"], dt)) for i in range(W)]
            avg = weighted_sum([x.reshape(-1) for x in xs], MUL_W, [v / N for v in n]).reshape(xs[0].shape)
            if k in params:
                p = state[k].clone().contiguous()
                first = k not in bufs
                if meta["server_momentum"] != 0 and first:
                    bufs[k] = torch.empty_like(p)
                sgd_apply(avg.contiguous(), p, bufs.get(k) if meta["server_momentum"] != 0 else None,
                          meta["server_lr"], meta["server_momentum"], 0.0, 0.0, False, first)
                new[k] = p
            else:
                new[k] = avg.to(state[k].dtype)  # load_state_dict copy_: float -> int64 truncates
        state = new
        outs.append(OrderedDict((k, v.cpu()) for k, v in state.items()))
    return outs


def fedopt_expected(meta, arrays):
    from golden_io import np_to_tensor
    return [OrderedDict((k, np_to_tensor(arrays[f"r{r}_y__{k}"], dt)) for k, dt in zip(meta["keys"], meta["dtypes"]))
            for r in range(len(meta["rounds"]))]


# ----------------------------------------------------------------------------- finite field (SecAgg)
MOD_FIRST, MOD_EACH, MOD_END, REAL_F64 = 1, 2, 4, 8


def sa_order_and_flags(uploaded):
    """SecAgg reconstruction (sa_fedml_aggregator.py:150-164): clients summed and the mod flags, given
    the per-client upload flags of the first-round active clients [0..N)."""
    order = [0] + [i for i in range(1, len(uploaded)) if uploaded[i]]
    return order, MOD_EACH | MOD_END | (MOD_FIRST if uploaded[0] else 0)


def finite_case_inputs(meta, arrays):
    """(clients as int64/float CPU tensors per key) for a finite-field fixture."""
    return client_dicts(meta, arrays)
