"""Read the committed golden vectors under tests/golden/ (written by tools/gen_golden.py).

Each case <name> has:
  <name>.in.jsonl.gz   MatchIn values as exchange_test.js / the generators send them (JSON lines)
  <name>.tape.txt.gz   MatchOut as consumer.js prints it: "<key> <value>" per forwarded record
  <name>.books.txt     sorted Books/Buckets/Orders store contents
  <name>.ledger.txt    sorted Balances/Positions store contents (when meta["ledger"])
  <name>.meta.json     how it was generated, engine mode, expected domain error if any
"""
import gzip
import json
import os

from kme.workloads import Orders

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def path(case, kind):
    return os.path.join(GOLDEN, {
        "in": f"{case}.in.jsonl.gz", "tape": f"{case}.tape.txt.gz", "books": f"{case}.books.txt",
        "ledger": f"{case}.ledger.txt", "meta": f"{case}.meta.json"}[kind])


def load_inputs(case):
    with open(path(case, "meta")) as f:
        meta = json.load(f)
    rows = []
    with gzip.open(path(case, "in"), "rt") as f:
        for line in f:
            d = json.loads(line)
            oid = d.get("oid", 0)
            rows.append((int(d.get("action", 0)), int(oid), int(d.get("aid", 0)), int(d.get("sid", 0)),
                         int(d.get("price", 0)), int(d.get("size", 0)), isinstance(oid, str)))
    return Orders.from_rows(rows), meta


def load_json_lines(case):
    with gzip.open(path(case, "in"), "rt") as f:
        return [l.rstrip("\n") for l in f]


def load_text(case, kind):
    p = path(case, kind)
    if p.endswith(".gz"):
        with gzip.open(p, "rt") as f:
            return f.read()
    with open(p) as f:
        return f.read()


def cases():
    if not os.path.isdir(GOLDEN):
        return []
    return sorted(f[: -len(".meta.json")] for f in os.listdir(GOLDEN) if f.endswith(".meta.json"))
