"""GPU tests of the drop-in front-end (vrpms_amd.solver): every algorithm
returns the handler result schema, and every reported duration equals the
spec oracle's duration of the returned routes."""
import itertools

import numpy as np
import pytest

from oracle import spec
from vrpms_amd import solver, synth

pytestmark = pytest.mark.gpu

KNOBS = {"sa": {"chains": 128, "steps": 600}, "ga": {"pop": 64, "iteration_count": 60},
         "aco": {"ants": 32, "iteration_count": 20}, "bf": {}}


def tsp_matrix(N=9, seed=3):
    rng = np.random.default_rng(seed)
    return synth.random_symmetric(N, rng)


@pytest.mark.parametrize("algo", ["bf", "sa", "ga", "aco"])
def test_solve_tsp_schema_and_cost(algo):
    D = tsp_matrix()
    customers = [1, 3, 4, 6, 7, 8]
    res = solver.solve_tsp(algo, D.tolist(), customers, 5, 30, seed=1, **KNOBS[algo])
    assert set(res) == {"duration", "vehicle"}
    v = res["vehicle"]
    assert v[0] == v[-1] == 5 and sorted(v[1:-1]) == customers
    assert res["duration"] == spec.eval_tsp(D[np.ix_(v[:-1], v[:-1])], list(range(1, len(v) - 1)), 30)
    if algo == "bf":
        best = min(sum(D[a, b] for a, b in zip((5,) + p, p + (5,)))
                   for p in itertools.permutations(customers))
        assert res["duration"] == best


def route_cost(D, tour, start):
    t = start
    for a, b in zip(tour, tour[1:]):
        t += int(D[(t // 60) % D.shape[0], a, b])
    return t - start


@pytest.mark.parametrize("algo", ["bf", "sa", "ga", "aco"])
def test_solve_vrp_schema_and_cost(algo):
    inst = synth.cvrp(8 if algo == "bf" else 30, 3, seed=4, slack=1.2)
    D = inst.durations
    locs = [{"id": 100 + i, "demand": int(inst.demand[i])} for i in range(inst.N)]
    ignored, completed = [102], [105]
    res = solver.solve_vrp(algo, D[0].tolist(), locs, inst.capacities.tolist(),
                           [0, 10, 20], ignored, completed, seed=2, **KNOBS[algo])
    assert set(res) == {"durationMax", "durationSum", "vehicles"}
    assert len(res["vehicles"]) == 3
    served = []
    for v, st in zip(res["vehicles"], [0, 10, 20]):
        assert v["tour"][0] == v["tour"][-1] == 0
        served += v["tour"][1:-1]
        assert v["duration"] == (route_cost(D, v["tour"], st) if len(v["tour"]) > 2 else 0)
    assert sorted(served) == [i for i in range(1, inst.N) if i not in (2, 5)]
    assert res["durationSum"] == sum(v["duration"] for v in res["vehicles"])
    assert res["durationMax"] == max(v["duration"] for v in res["vehicles"])


def test_solve_vrp_bf_is_optimal_over_giant_tours():
    inst = synth.cvrp(7, 2, seed=6, slack=1.3)
    locs = [{"id": i, "demand": int(inst.demand[i])} for i in range(inst.N)]
    res = solver.solve_vrp("bf", inst.durations[0], locs, inst.capacities, inst.start_times)
    best = min(spec.eval_cvrp(inst.durations, p, inst.demand, inst.capacities,
                              inst.start_times)["key"]
               for p in itertools.permutations(range(1, 8)))
    assert spec.pack_key(0, res["durationSum"], res["durationMax"]) == best


def test_time_dependent_vrp():
    inst = synth.td_cvrp(25, 3, seed=2)
    locs = [{"id": i, "demand": int(inst.demand[i])} for i in range(inst.N)]
    res = solver.solve_vrp("sa", inst.durations.tolist(), locs, inst.capacities.tolist(),
                           inst.start_times.tolist(), seed=3, chains=64, steps=400)
    for v, st in zip(res["vehicles"], inst.start_times):
        if len(v["tour"]) > 2:
            assert v["duration"] == route_cost(inst.durations, v["tour"], int(st))


def test_solve_vrp_problem_default_and_bf_errors():
    r = solver.solve_vrp_problem(seed=4, chains=64, steps=300)
    assert set(r) == {"tour", "total_time", "unvisited", "date"}
    assert r["tour"][0] == r["tour"][-1] == 0 and sorted(r["tour"][1:-1]) == list(range(1, 15))
    assert r["unvisited"] == []
    cap = solver.BF_MAX_CUSTOMERS
    with pytest.raises(ValueError, match="brute force"):
        solver.solve_tsp("bf", tsp_matrix(cap + 2).tolist(), list(range(1, cap + 2)), 0)
    # at the cap (13! = 6.2 G tours) the exhaustive optimum is below any SA tour
    D = tsp_matrix(cap + 1).tolist()
    bf = solver.solve_tsp("bf", D, list(range(1, cap + 1)), 0)
    sa = solver.solve_tsp("sa", D, list(range(1, cap + 1)), 0, chains=64, steps=500)
    assert sorted(bf["vehicle"][1:-1]) == list(range(1, cap + 1))
    assert bf["duration"] <= sa["duration"]
    with pytest.raises(ValueError, match="unknown algorithm"):
        solver.solve_tsp("tabu", tsp_matrix().tolist(), [1, 2], 0)
    # an hour-indexed matrix keeps the lower cap (every edge priced at its hour)
    import numpy as np
    td = np.stack([tsp_matrix(13)] * 24)
    with pytest.raises(ValueError, match=f"at most {solver.BF_MAX_CUSTOMERS_TD}"):
        solver.solve_tsp("bf", td.tolist(), list(range(1, 13)), 0)


def test_tiny_instances():
    D = tsp_matrix(3)
    assert solver.solve_tsp("sa", D.tolist(), [], 1) == {"duration": int(D[1, 1]),
                                                        "vehicle": [1, 1]}
    r = solver.solve_tsp("ga", D.tolist(), [2], 0, pop=8, iteration_count=2)
    assert r == {"duration": int(D[0, 2] + D[2, 0]), "vehicle": [0, 2, 0]}


@pytest.mark.parametrize("algo", ["sa", "ga", "aco"])
def test_solve_vrp_island_model_across_devices(algo):
    """devices=[0, 0]: the in-process island model (one island per listed
    device, elites exchanged device to device by islands.exchange_local) on
    the one-GPU box -- the same code path as a node's distinct GPUs.  The
    answer keeps the schema and every reported duration is the spec's."""
    inst = synth.cvrp(30, 3, seed=5, slack=1.2)
    D = inst.durations
    locs = [{"id": i, "demand": int(inst.demand[i])} for i in range(inst.N)]
    res = solver.solve_vrp(algo, D[0].tolist(), locs, inst.capacities.tolist(), [0, 0, 0], [],
                           [], seed=3, devices=[0, 0], **KNOBS[algo])
    served = []
    for v in res["vehicles"]:
        served += v["tour"][1:-1]
        assert v["duration"] == (route_cost(D, v["tour"], 0) if len(v["tour"]) > 2 else 0)
    assert sorted(served) == list(range(1, inst.N))
    assert res["durationSum"] == sum(v["duration"] for v in res["vehicles"])


def test_exchange_local_gives_every_island_the_global_elites():
    """islands.exchange_local == pack every island, merge all messages in
    island order, inject: after it each island's worst chains hold the same
    E global best tours (SA pools on one device standing in for two)."""
    import torch
    from vrpms_amd import islands, runners
    from vrpms_amd.core import CVRP
    inst = synth.cvrp(40, 4, seed=6, slack=1.2)
    ctx = solver.context(0)
    ctx.set_instance(CVRP, inst.durations, inst.demand, inst.capacities, inst.start_times)
    rs = [runners.SARunner(ctx, inst.n, chains=64, seed=s, total_steps=200) for s in (1, 2)]
    for r in rs:
        r.epoch(50)
    E = 4
    msgs = torch.cat([ctx.island_pack(*r.src(), E) for r in rs])
    want_t, want_k = ctx.island_merge(msgs, 2, E, rs[0].n)
    islands.exchange_local(rs, E)
    for r in rs:
        keys = r.cur_key.cpu()
        for e in range(E):
            hit = (keys == want_k[e].cpu()).nonzero().flatten().tolist()
            assert any(torch.equal(r.cur[i].cpu(), want_t[e].cpu()) for i in hit)
