"""GPU parity at bench-like scale: hundreds to tens of thousands of symbol groups matched in one
launch, epochs of 2^18 records, every epoch's MatchOut tape byte-identical to the oracle's and the
final book stores equal.

The small parity tests (test_gpu_parity.py) touch a few hundred node slots; at this scale the
slots run into the tens of thousands, free-list blocks get recycled across batches, and
cancels hit orders that were swept earlier in the same epoch -- the combination that exposed a
stale-node acceptance in k_match's batch cancel prefetch (a freed slot hosting a free-list block
has a slot id in word 12, whose bit 11 was packed over the prefetch's `ok` bit).
"""
import pytest

from kme import workloads as W

pytestmark = pytest.mark.gpu

E = 1 << 18


def _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, light_max, epoch=E):
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1,
                                                max_epoch=max(epoch, len(setup)), max_resting=1 << 22,
                                                max_trades=2 * epoch + (1 << 16), max_accounts=n_acc,
                                                light_max=light_max))
    o = oracle_mod.Oracle()
    parts = [setup] + [stream.slice(a, min(len(stream), a + epoch)) for a in range(0, len(stream), epoch)]
    for k, part in enumerate(parts):
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        if got != want:
            la, lb = got.splitlines(), want.splitlines()
            j = next((j for j, (x, y) in enumerate(zip(la, lb)) if x != y), min(len(la), len(lb)))
            pytest.fail(f"epoch {k}: line {j}: got {la[j] if j < len(la) else None!r} "
                        f"want {lb[j] if j < len(lb) else None!r}")
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


@pytest.mark.parametrize("light_max", [-1, 0])
def test_c5_cancel_replace_at_scale(kme_mod, oracle_mod, light_max):
    """C5 (1,024 symbols, 4,096 accounts): cancels of orders swept earlier in the epoch."""
    n_sym, n_acc, n = 1024, 4096, 6 * E
    stream = W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1),
                           transfers_per_account=W.funded_transfers_needed(n, n_acc, big=True))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, light_max)


def test_c3_uniform_at_scale(kme_mod, oracle_mod):
    """C3's shape (65,536 symbols and accounts): light groups in lanes, busy ones in wavefronts."""
    n_sym, n_acc, n = 65536, 65536, 4 * E
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


def test_c2_uniform_at_scale(kme_mod, oracle_mod):
    """C2's shape (1,024 symbols): every group busy, one wavefront each."""
    n_sym, n_acc, n = 1024, 4096, 4 * E
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1001)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


def test_c4_zipf_at_scale(kme_mod, oracle_mod):
    """C4's shape (Zipf(1.1) over 8,192 symbols): hot books thousands of orders deep."""
    n_sym, n_acc, n = 8192, 16384, 2 * E
    stream = W.zipf(n, n_symbols=n_sym, n_accounts=n_acc, seed=1002)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)



def test_n8_shard_shape_at_scale(kme_mod, oracle_mod):
    """The per-GPU shard of C3 at N = 8 (8,192 symbols), 2^21-record epochs: 256 records per group
    per epoch, every group busy (one wavefront each), several record batches per group."""
    n_sym, n_acc, n = 8192, 65536, 1 << 22
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1003)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0, epoch=1 << 21)
