"""Pins the C1 input stream to the reference's own generator (round-3 verdict, next-round item 9).

Runs /root/reference/exchange_test.js -- read where it lies, never copied -- under this container's
node (v12) with three stand-ins: a local `kafkajs` module whose producer records each message value
(the script's only use of the broker), a silent console.log, and Math.random served from a seeded
stream of doubles, the same stream kme.workloads._JsRandom(seed) draws from.  The producer stops the
script after the requested number of messages (exchange_test.js catches the error and exits), and the
recorded MatchIn values are written as a gzipped JSON-lines fixture.  tests/test_workloads.py requires
kme.workloads.exchange_test(n, seed) to reproduce the fixture record for record.

This pins the inputs only (what the reference's harness sends); matching parity stays with the oracle.

usage: python tools/gen_exchange_test_fixture.py [n_events] [seed] [out.jsonl.gz]
"""
import gzip
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference/exchange_test.js"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r"""
// kafkajs stand-in: a producer that records what exchange_test.js sends (no broker)
const fs = require('fs');
const limit = parseInt(process.env.KME_FIXTURE_LIMIT, 10);
const out = process.env.KME_FIXTURE_OUT;
const sent = [];
function dump() { fs.writeFileSync(out, sent.join('\n') + '\n'); }
class Kafka {
  constructor(cfg) { this.cfg = cfg; }
  producer() {
    return {
      connect: async () => {},
      disconnect: async () => { dump(); },
      send: async (msg) => {
        if (sent.length >= limit) { dump(); throw new Error('fixture complete'); }
        for (const m of msg.messages) sent.push(m.value);
        return [{topicName: msg.topic, partition: 0, errorCode: 0}];
      },
    };
  }
}
module.exports = {Kafka};
"""

PRELUDE = r"""
// Math.random from the seeded stream of doubles (float64 little endian); console.log silenced
const fs = require('fs');
const buf = fs.readFileSync(process.env.KME_FIXTURE_RANDOM);
const r = new Float64Array(buf.buffer, buf.byteOffset, buf.length / 8);
let at = 0;
Math.random = function () {
  if (at >= r.length) throw new Error('random stream exhausted');
  return r[at++];
};
console.log = function () {};
require(process.env.KME_FIXTURE_SCRIPT);
"""


def generate(n_events: int, seed: int) -> list:
    n_msgs = 10 * 2 + 3 + n_events          # exchange_test.js:23-36: accounts, transfers, symbols, events
    with tempfile.TemporaryDirectory() as tmp:
        mods = os.path.join(tmp, "node_modules", "kafkajs")
        os.makedirs(mods)
        with open(os.path.join(mods, "index.js"), "w") as f:
            f.write(STUB)
        rnd = os.path.join(tmp, "random.f64")
        # the doubles kme.workloads._JsRandom(seed) yields (PCG64, one 64-bit draw per double)
        np.random.Generator(np.random.PCG64(seed)).random(12 * n_msgs + 4096).astype("<f8").tofile(rnd)
        prelude = os.path.join(tmp, "prelude.js")
        with open(prelude, "w") as f:
            f.write(PRELUDE)
        out = os.path.join(tmp, "sent.jsonl")
        env = dict(os.environ, NODE_PATH=os.path.join(tmp, "node_modules"), KME_FIXTURE_LIMIT=str(n_msgs),
                   KME_FIXTURE_OUT=out, KME_FIXTURE_RANDOM=rnd, KME_FIXTURE_SCRIPT=REF)
        subprocess.run(["node", prelude], check=True, env=env, timeout=600)
        with open(out) as f:
            lines = [ln for ln in f.read().split("\n") if ln]
    assert len(lines) == n_msgs, (len(lines), n_msgs)
    return lines


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "tests", "golden", f"exchange_test_js_n{n}_s{seed}.jsonl.gz")
    lines = generate(n, seed)
    with gzip.open(out, "wt") as f:
        f.write("\n".join(lines) + "\n")
    print(f"{out}: {len(lines)} MatchIn values from {REF} under node {subprocess.check_output(['node', '--version']).decode().strip()}")


if __name__ == "__main__":
    main()
