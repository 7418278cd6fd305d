#!/usr/bin/env python3
"""Capture what the reference pins as JSON fixtures.

Run in the build container only (it imports /root/reference read-only;
the GPU box never sees the reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_reference_fixtures.py

Shims (the reference's own code is executed unmodified):
  * `dotenv` -- python-dotenv is not installed; load_dotenv becomes a no-op.
  * `supabase` -- the remote DB is unreachable offline; an in-process fake
    returns configured rows for locations/durations and records inserts.
Captured:
  remove_unused_locations cases        api/helpers.py:11-13
  parse_* outputs + error lists        api/parameters.py:4-56, api/helpers.py:5-8
  wire responses of all 8 endpoints    api/{tsp,vrp}/{bf,ga,sa,aco}/index.py
  solver stub shapes under random.seed src/solver.py:7-27 (date masked)
"""
import importlib
import io
import json
import os
import random
import sys
import types

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_fixtures.json")
sys.dont_write_bytecode = True


def install_shims(db):
    d = types.ModuleType("dotenv")
    d.load_dotenv = lambda *a, **k: None
    sys.modules["dotenv"] = d

    class Result:
        def __init__(self, data):
            self.data = data

    class Query:
        def __init__(self, table):
            self.table, self.filters, self.payload = table, {}, None

        def select(self, *_a):
            return self

        def eq(self, col, val):
            self.filters[col] = val
            return self

        def insert(self, payload):
            self.payload = payload
            return self

        def execute(self):
            if self.payload is not None:
                db["inserts"].append({"table": self.table, "data": self.payload})
                return Result([self.payload])
            rows = db["tables"].get(self.table, {})
            key = self.filters.get("id")
            return Result([rows[key]] if key in rows else [])

    class User:
        def model_dump(self):
            return {"user": {"email": "tester@example.com"}}

    class Auth:
        def set_session(self, **_k):
            db["sessions"] += 1

        def get_user(self):
            return User()

    class Client:
        def __init__(self):
            self.auth = Auth()

        def table(self, t):
            return Query(t)

    sb = types.ModuleType("supabase")
    cl = types.ModuleType("supabase.client")
    cl.create_client = lambda url, key, options=None: Client()
    cl.Client = Client
    lib = types.ModuleType("supabase.lib")
    co = types.ModuleType("supabase.lib.client_options")
    co.ClientOptions = lambda **k: k
    for name, mod in {"supabase": sb, "supabase.client": cl, "supabase.lib": lib,
                      "supabase.lib.client_options": co}.items():
        sys.modules[name] = mod


def call(handler_cls, method, body=None):
    h = handler_cls.__new__(handler_cls)
    raw = json.dumps(body).encode() if body is not None else b""
    h.rfile = io.BytesIO(raw)
    h.wfile = io.BytesIO()
    h.headers = {"Content-Length": str(len(raw))}
    h.request_version = "HTTP/1.0"
    h.requestline = f"{method} / HTTP/1.0"
    h.command = method
    h.client_address = ("127.0.0.1", 0)
    h.log_message = lambda *a, **k: None
    getattr(h, "do_" + method)()
    text = h.wfile.getvalue().decode()
    head, _, payload = text.partition("\r\n\r\n")
    lines = head.split("\r\n")
    headers = [ln for ln in lines[1:] if not ln.startswith(("Date:", "Server:"))]
    return {"status_line": lines[0], "headers": headers, "body": payload}


def main():
    db = {"tables": {}, "inserts": [], "sessions": 0}
    install_shims(db)
    sys.path.insert(0, REF)
    helpers = importlib.import_module("api.helpers")
    params = importlib.import_module("api.parameters")
    solver = importlib.import_module("src.solver")
    fx = {"generator": "tests/golden/gen_reference_fixtures.py", "reference": "metehkaya/vrpms"}

    locs = [{"id": i, "name": f"L{i}"} for i in range(6)]
    cases = [(locs, [2], [4]), (locs, [], []), (locs, [0], []), (locs, [9], [1, 3, 5]),
             ([{"id": "a"}, {"id": "b"}], ["b"], [])]
    fx["remove_unused_locations"] = [
        {"locations": l, "ignored": i, "completed": c,
         "result": helpers.remove_unused_locations(l, i, c)} for l, i, c in cases]

    full_vrp = {"solutionName": "n", "solutionDescription": "d", "locationsKey": 1,
                "durationsKey": 2, "capacities": [5, 5], "startTimes": [0, 30],
                "ignoredCustomers": [], "completedCustomers": [], "multiThreaded": False,
                "randomPermutationCount": 10, "iterationCount": 5}
    full_tsp = {"solutionName": "n", "solutionDescription": "d", "locationsKey": 1,
                "durationsKey": 2, "customers": [1, 2, 3], "startNode": 0, "startTime": 0}
    parse = {}
    for name in ["parse_common_vrp_parameters", "parse_vrp_ga_parameters",
                 "parse_vrp_sa_parameters", "parse_vrp_aco_parameters",
                 "parse_common_tsp_parameters", "parse_tsp_ga_parameters",
                 "parse_tsp_sa_parameters", "parse_tsp_aco_parameters"]:
        fn = getattr(params, name)
        out = {}
        for label, body in [("empty", {}), ("vrp_full", full_vrp), ("tsp_full", full_tsp),
                            ("falsy", {k: 0 for k in full_vrp})]:
            errs = []
            out[label] = {"params": fn(dict(body), errs), "errors": errs}
        parse[name] = out
    fx["parse"] = parse

    random.seed(7)
    fx["calculate_duration"] = [solver.calculate_duration("A", "B") for _ in range(3)]
    stub = []
    for s in range(3):
        random.seed(s)
        r = solver.solve_vrp_problem()
        r["date"] = "<masked>"
        stub.append(r)
    fx["solve_vrp_problem"] = stub

    # wire contract: a 4-node instance in the fake DB
    db["tables"]["locations"] = {1: {"id": 1, "locations": [{"id": i} for i in range(4)]}}
    db["tables"]["durations"] = {2: {"id": 2, "matrix": [[0, 5, 6, 7], [5, 0, 8, 9],
                                                          [6, 8, 0, 4], [7, 9, 4, 0]]}}
    wire = {}
    for prob in ["tsp", "vrp"]:
        for algo in ["bf", "ga", "sa", "aco"]:
            mod = importlib.import_module(f"api.{prob}.{algo}.index")
            body = dict(full_vrp if prob == "vrp" else full_tsp)
            ent = {"GET": call(mod.handler, "GET"),
                   "POST_empty": call(mod.handler, "POST", {}),
                   "POST_full": call(mod.handler, "POST", body),
                   "POST_missing_db": call(mod.handler, "POST", {**body, "durationsKey": 99})}
            db["inserts"].clear()
            ent["POST_auth"] = call(mod.handler, "POST", {**body, "auth": "jwt",
                                                          "ignoredCustomers": [2]}
                                    if prob == "vrp" else {**body, "auth": "jwt"})
            ent["POST_auth_insert"] = db["inserts"][:]
            if hasattr(mod.handler, "do_OPTIONS"):
                ent["OPTIONS"] = call(mod.handler, "OPTIONS")
            wire[f"{prob}/{algo}"] = ent
    fx["wire"] = wire
    with open(OUT, "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True, default=str)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
