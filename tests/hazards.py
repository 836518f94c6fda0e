"""Hand-built record streams that force each semantic hazard of SURVEY.md §8.1 (H1-H9).

Each entry: name -> (rows, mode_ok) where rows are (action, oid, aid, sid, price, size) tuples and
`funded_ok` says whether the stream is legal in FUNDED mode (no ledger-dependent acceptance).
"""
from kme.workloads import (ADD_SYMBOL, BUY, CANCEL, CREATE_BALANCE, PAYOUT, REMOVE_SYMBOL, SELL, TRANSFER,
                           Orders)

BIG = 2**31 - 1


def _setup(accounts=(1, 2, 3, 4), sids=(0, 1, 2), fund=BIG):
    rows = []
    for a in accounts:
        rows.append((CREATE_BALANCE, 0, a, 0, 0, 0))
        rows.append((TRANSFER, 0, a, 0, 0, fund))
    for s in sids:
        rows.append((ADD_SYMBOL, 0, 0, s, 0, 0))
    return rows


def streams():
    S = {}
    # H3: BUY taker exactly exhausts the head maker while another maker waits at the taker's price
    S["zero_trade_same_level"] = _setup() + [
        (SELL, 11, 1, 1, 50, 10), (SELL, 12, 2, 1, 50, 5), (BUY, 13, 3, 1, 50, 10)]
    # H3: SELL taker always tests maker.price >= P; exact fill then the next (lower) level still >= P
    S["zero_trade_next_level"] = _setup() + [
        (BUY, 21, 1, 2, 60, 7), (BUY, 22, 2, 2, 55, 9), (SELL, 23, 3, 2, 50, 7)]
    # BUY exact fill, level exhausted, next ask above the limit -> zero trade with its head
    S["zero_trade_buy_next_level_above"] = _setup() + [
        (SELL, 31, 1, 1, 40, 8), (SELL, 32, 2, 1, 45, 3), (BUY, 33, 3, 1, 42, 8)]
    # size-0 orders: rest with size 0 on an empty book, then get consumed with zero trades
    S["size_zero"] = _setup() + [
        (BUY, 41, 1, 1, 50, 0), (BUY, 42, 2, 1, 50, 0), (SELL, 43, 3, 1, 50, 0), (SELL, 44, 3, 1, 49, 5),
        (BUY, 45, 4, 1, 55, 3)]
    # H4: sid 0 is one shared book; a BUY matches whatever sits at the minimum, even a bid
    S["sid0_shared_book"] = _setup() + [
        (BUY, 51, 1, 0, 40, 5), (SELL, 52, 2, 0, 60, 5), (BUY, 53, 3, 0, 45, 3), (SELL, 54, 4, 0, 58, 2),
        (BUY, 55, 1, 0, 59, 9), (SELL, 56, 2, 0, 1, 4)]
    # negative sid addresses the opposite side of |sid|
    S["negative_sid"] = _setup() + [
        (BUY, 61, 1, -1, 50, 5), (SELL, 62, 2, 1, 55, 5), (BUY, 63, 3, 1, 56, 2), (SELL, 64, 4, -1, 45, 9)]
    # cancels: head / middle / tail / only, wrong aid, unknown oid, filled order, in-epoch order
    S["cancels"] = _setup() + [
        (BUY, 71, 1, 1, 40, 5), (BUY, 72, 2, 1, 40, 6), (BUY, 73, 3, 1, 40, 7), (BUY, 74, 4, 1, 40, 8),
        (CANCEL, 72, 2, 0, 0, 0), (CANCEL, 71, 1, 0, 0, 0), (CANCEL, 74, 4, 0, 0, 0), (CANCEL, 73, 1, 0, 0, 0),
        (CANCEL, 999, 1, 0, 0, 0), (SELL, 75, 2, 1, 40, 7), (CANCEL, 73, 3, 0, 0, 0), (BUY, 76, 1, 1, 33, 2),
        (CANCEL, 76, 1, 0, 0, 0), (SELL, 77, 1, 2, 70, 3), (BUY, 78, 2, 2, 71, 1), (CANCEL, 77, 1, 0, 0, 0),
        (CANCEL, 77, 1, 0, 0, 0)]
    # multi-level sweep with partial fills on both ends
    S["sweep"] = _setup() + [
        (SELL, 81, 1, 1, 50, 4), (SELL, 82, 2, 1, 51, 4), (SELL, 83, 3, 1, 51, 2), (SELL, 84, 4, 1, 53, 9),
        (SELL, 85, 1, 1, 60, 1), (BUY, 86, 2, 1, 53, 13), (BUY, 87, 3, 1, 70, 20), (SELL, 88, 4, 1, 10, 3)]
    # symbol admin: duplicate ADD_SYMBOL, REMOVE_SYMBOL absent (accepted) / existing empty (rejected),
    # orders on an absent symbol, unknown action
    S["symbol_admin"] = _setup(sids=(1,)) + [
        (ADD_SYMBOL, 0, 0, 1, 0, 0), (ADD_SYMBOL, 0, 0, -1, 0, 0), (REMOVE_SYMBOL, 0, 0, 5, 0, 0),
        (REMOVE_SYMBOL, 0, 0, 1, 0, 0), (BUY, 91, 1, 5, 50, 5), (ADD_SYMBOL, 0, 0, 5, 0, 0),
        (BUY, 92, 1, 5, 50, 5), (REMOVE_SYMBOL, 0, 0, -5, 0, 0), (42, 0, 0, 0, 0, 0), (SELL, 93, 2, 5, 40, 9)]
    # price levels across the lsb/msb word boundary (62 / 63 / 64) and the top level 125
    S["word_boundary"] = _setup() + [
        (SELL, 101, 1, 1, 63, 2), (SELL, 102, 2, 1, 62, 2), (SELL, 103, 3, 1, 64, 2), (SELL, 104, 4, 1, 100, 2),
        (BUY, 105, 1, 1, 63, 3), (BUY, 106, 2, 1, 100, 5), (BUY, 107, 3, 1, 0, 1), (BUY, 108, 4, 1, 62, 1),
        (SELL, 109, 1, 1, 61, 4)]
    # prices above 100 (sell risk turns into a credit) up to the top usable level 125 (EXACT only)
    S["top_levels"] = _setup(fund=10_000) + [
        (SELL, 141, 1, 1, 125, 2), (SELL, 142, 2, 1, 110, 2), (BUY, 143, 3, 1, 120, 3), (BUY, 144, 4, 1, 125, 5),
        (SELL, 145, 1, 1, 101, 9), (BUY, 146, 2, 1, 124, 1), (SELL, 147, 3, 1, 124, 1)]
    # ---- ledger-coupled streams (EXACT mode only)
    # H1: balance runs dry -> REJECT; refunds from fills and cancels; transfers in and out
    S["ledger_gate"] = _setup(fund=1000) + [
        (BUY, 111, 1, 1, 50, 10), (BUY, 112, 1, 1, 50, 11), (BUY, 113, 1, 1, 50, 10),
        (SELL, 114, 2, 1, 40, 4), (CANCEL, 111, 1, 0, 0, 0), (BUY, 115, 1, 1, 50, 10),
        (TRANSFER, 0, 1, 0, 0, -400), (TRANSFER, 0, 1, 0, 0, -1), (TRANSFER, 0, 9, 0, 0, 5),
        (CREATE_BALANCE, 0, 1, 0, 0, 0), (SELL, 116, 3, 1, 30, 30), (BUY, 117, 9, 1, 50, 1)]
    # H2: positions written under the VALUE as key; a zero fill creates (0,0) entries that clobber
    # account 0 / symbol 0; sells against long positions use `available`
    S["positions_h2"] = _setup(accounts=(0, 1, 2, 3), fund=100000) + [
        (SELL, 121, 1, 0, 50, 10), (SELL, 122, 2, 0, 50, 5), (BUY, 123, 3, 0, 50, 10),
        (BUY, 124, 0, 0, 60, 5), (SELL, 125, 3, 0, 40, 6), (BUY, 126, 1, 1, 44, 1), (SELL, 127, 2, 1, 44, 1),
        (SELL, 128, 3, 0, 45, 4), (CANCEL, 128, 3, 0, 0, 0), (BUY, 129, 2, 1, 50, 1), (SELL, 130, 1, 1, 50, 1)]
    # PAYOUT (action 200) on an absent symbol settles positions with key lsb == sid; on an existing
    # empty book it is a no-op; its result is always REJECT
    S["payout"] = _setup(accounts=(1, 2), sids=(1,), fund=100000) + [
        (BUY, 131, 1, 1, 50, 3), (SELL, 132, 2, 1, 50, 3), (PAYOUT, 0, 0, 7, 0, 97), (PAYOUT, 0, 0, 1, 0, 97)]
    return S


FUNDED_OK = {"zero_trade_same_level", "zero_trade_next_level", "zero_trade_buy_next_level_above", "size_zero",
             "sid0_shared_book", "negative_sid", "cancels", "sweep", "symbol_admin", "word_boundary"}

# Streams where the reference throws / never returns (KME_E_DOMAIN with the given detail).
def domain_streams():
    D = {}
    # H5: 48 contiguous bid levels 0..47 -> getLastSetBitPos overshoots to 48 (empty) -> NPE
    rows = _setup()
    for p in range(48):
        rows.append((BUY, 1000 + p, 1, 1, p, 1))
    rows.append((SELL, 2000, 2, 1, 0, 1))
    D["log10_overshoot"] = (rows, 2)
    # price 126 is msb bit 63: getLastSetBitPos(negative) = 0 -> bucket 63 (empty) -> NPE
    D["price_126"] = (_setup() + [(BUY, 3000, 1, 1, 126, 1), (SELL, 3001, 2, 1, 100, 1)], 2)
    # removeAllOrders on a non-empty book never terminates
    D["remove_nonempty"] = (_setup() + [(BUY, 4000, 1, 1, 50, 1), (REMOVE_SYMBOL, 0, 0, 1, 0, 0)], 5)
    return D


def as_orders(rows) -> Orders:
    return Orders.from_rows(rows)
