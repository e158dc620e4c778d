"""Exchange of the distributed Table layer (capf_amd/dist_table.py) over the
numpy oracle tables — test infrastructure: the CPU tests run the product's
DistTable operator rules on OracleTable shards with gloo, rows routed by the
numpy restatement of csrc/shuffle.hip (oracle/route.py) and moved as pickled
slices (all_gather_object)."""
import numpy as np
import torch
import torch.distributed as dist

from capf_amd.expr import T_BOOL, T_FLOAT, T_NULL, T_STRING
from oracle import route
from oracle.table_np import Col, OracleTable, _empty_vals

_KIND = {T_FLOAT: "float", T_BOOL: "bool", T_STRING: "str", T_NULL: "null"}


def oracle_route_owners(table, keys, parts):
    cols = [table._cols[k] for k in keys[:8]]
    bits = [route.key_bits(_KIND.get(c.t, "int"), c.v, c.ok) for c in cols]
    return route.owners(bits, table.size, parts)


def _concat(tables, order, types):
    cols = {}
    for c, t0 in zip(order, types):
        parts = [tb._cols[c] for tb in tables]
        t = next((p.t for p in parts if p.t != T_NULL), t0)
        vs = [p.v if p.t == t else _empty_vals(t, len(p.ok)) for p in parts]
        cols[c] = Col(t, np.concatenate(vs) if vs else _empty_vals(t, 0),
                      np.concatenate([p.ok for p in parts]) if parts else np.zeros(0, bool))
    return OracleTable(order, cols, sum(tb.size for tb in tables))


class OracleExchange:
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_sum(self, v):
        t = torch.tensor([int(v)], dtype=torch.int64)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def all_max_vec(self, vals):
        t = torch.tensor(list(vals) or [0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.tolist()[:len(vals)]

    def all_gather_obj(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def route(self, table, keys):
        own = oracle_route_owners(table, list(keys), self.world)
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=self.world).tolist()
        return table._take(order), counts

    def shuffle(self, table, keys):
        routed, counts = self.route(table, keys)
        return self.send(routed, counts)

    def own_share(self, table, keys):
        routed, counts = self.route(table, keys)
        off = sum(counts[:self.rank])
        return routed._take(np.arange(off, off + counts[self.rank]))

    def to_root(self, table):
        return self.send(table, [table.size if p == 0 else 0 for p in range(self.world)])

    def replicate(self, table):
        return self.send(table, [table.size] * self.world, repeat=True)

    def send(self, table, counts, repeat=False):
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        if repeat:
            slices = [table] * self.world
        else:
            slices = [table._take(np.arange(off[p], off[p + 1])) for p in range(self.world)]
        got = self.all_gather_obj(slices)
        mine = [g[self.rank] for g in got]
        order = table.physicalColumns
        return _concat(mine, order, [table.capf_type(c) for c in order])


def oracle_count_copies(dsession, rt, n, lo, compact=True):
    """Oracle stand-in for the GPU copies of dist_node_partitioned_graph: this
    rank's partial Σ_{b owned} in[b]·out[b] − owned self-loops with b owned
    when (b − lo) mod G = rank (any partition of the node ids sums to the
    count), from the full rel table every rank holds."""
    src = np.asarray(rt.table.column_values(rt.src_col), dtype=np.int64) - lo
    dst = np.asarray(rt.table.column_values(rt.dst_col), dtype=np.int64) - lo
    world, rank = dsession.world, dsession.rank
    calls = oracle_count_copies.calls

    def partial():
        calls.append(rank)
        own = np.arange(n) % world == rank
        ins = np.bincount(dst, minlength=n)
        outs = np.bincount(src, minlength=n)
        loops = int(((src == dst) & own[src]).sum())
        return int((ins[own].astype(object) * outs[own].astype(object)).sum()) - loops
    return lambda: dsession.ex.all_sum(partial())


oracle_count_copies.calls = []
