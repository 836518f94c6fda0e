// GpuMatchingEngine -- the MI355X matching engine behind the reference's Processor interface, the
// swap at the topology (KProcessor.java:52-57):
//
//     .addProcessor("MatchingEngine", GpuMatchingEngine::new, "Source")
//     .addStateStore(GpuMatchingEngine.commitHook(), "MatchingEngine")
//     .addStateStore(GpuMatchingEngine.commitLog(), "MatchingEngine")
//
// Like the reference's MatchingEngine (KP:63) it is a Processor<String, Order> over the reference's
// own top-level Order class (KP:449-475), in the same (default) package; it uses only Order's public
// fields and its six-argument creator (KP:463-465).  tests/test_java_processor.py holds this file to
// KProcessor.java's declarations.
//
// Contract kept from MatchingEngine.process (KP:96-126): for every input record the processor
// forwards ("IN", order), then the maker and the taker fill of each trade (keyed "OUT", KP:272-273),
// then ("OUT", order) -- same order, same field values.  The difference is timing: records are
// buffered into an epoch and forwarded when the epoch completes.
//
// Path at rate (include/kme.h, "Host epochs at device rate"): two slots of direct ByteBuffers over
// native, registered memory (kme_jni.c allocates them) hold an epoch's Order columns (native byte
// order) and the MatchOut rows that come back, so an epoch crosses PCIe straight from and to them.
// While the GPU runs epoch k, process() fills the other slot; the wall-clock punctuator polls (never
// blocks) and forwards a finished epoch, and sends a partly filled one so that latency stays bounded.
//
// Commit and restart (INTEGRATION.md §3; the reference keeps its state in changelogged stores,
// KP:30-49, runs at least once, KP:29, and commits after every record, KP:125).  Kafka Streams
// commits the consumed offset of every record process() has returned from, and flushes the task's
// state stores first.  The commit hook is such a store: its flush() is this processor's commit
// point -- the partly filled epoch is submitted, every epoch in flight is completed (its rows kept,
// forwarded at the next process() or punctuation: forwarding is not possible inside a store flush),
// and one file written atomically holds the device state after the last record taken (its Kafka
// offset) and the rows not yet forwarded.  init() restores that file, forwards those rows first, and
// skips re-delivered records at or below the offset.  A record whose offset Kafka committed is
// therefore either forwarded or in the checkpoint; output forwarded after a checkpoint may be
// forwarded again after a crash (at least once, as the reference).
//
// The file lives in the task's local state directory; the state itself follows the task through the
// commit log, a changelogged key-value store (logging on, as the reference's five stores, KP:30-49):
// each commit point puts the file's chunks that changed since the last commit (fixed-size chunks keyed
// by index and content hash: a chunk another record still names is never overwritten) and then one
// record -- the checkpoint's generation, offset, size, digest and the hash of every chunk -- and Kafka
// Streams sends them to the changelog before it commits the offsets.  init() reads that record
// (restored from the changelog wherever the task runs): a local file that is the committed one is
// restored; otherwise (a moved task's empty state directory, an older or foreign file) the file is
// rebuilt from the changelogged chunks and restored; a record whose chunks are not all there, and no
// local file that is the committed one or newer, is refused instead of starting from an empty book at
// a committed offset.  A file newer than the record (a crash between the file's rename and the
// changelog write; Kafka then re-delivers from the older commit) is taken when the record's chunks are
// incomplete.
//
// Faults: the records before a fault took effect and are forwarded (as the reference's per-record
// commit would have, KP:97, 124-125); then the processor fails like the reference's stream thread.
// The default flags (EXACT_LEDGER | SERIAL_FALLBACK) give the reference's result for every record it
// takes -- any price and size, any account id, any symbol id below 2^55 (sparse ones up to the
// configured 4,096), the epochs the parallel path cannot prove or stage running on the serial engine
// (include/kme.h) -- so KME_E_UNFUNDED cannot occur; the faults left are the reference's own (its NPEs,
// a removeAllOrders that never returns) and capacities.  In a configuration without SERIAL_FALLBACK
// KME_E_UNFUNDED is fatal here too (its records were not processed, and a processor cannot hand
// records back to Kafka).
import java.io.File;
import java.io.FileOutputStream;
import java.io.IOException;
import java.io.RandomAccessFile;
import java.io.UncheckedIOException;
import java.nio.ByteBuffer;
import java.nio.file.Files;
import java.nio.file.StandardCopyOption;
import java.nio.ByteOrder;
import java.time.Duration;
import java.util.Collections;
import java.util.Map;

import org.apache.kafka.common.serialization.Serdes;
import org.apache.kafka.streams.processor.Processor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.PunctuationType;
import org.apache.kafka.streams.processor.StateStore;
import org.apache.kafka.streams.state.KeyValueStore;
import org.apache.kafka.streams.state.StoreBuilder;
import org.apache.kafka.streams.state.Stores;

public final class GpuMatchingEngine implements Processor<String, Order> {
    static { System.loadLibrary("kme_jni"); }

    // include/kme.h
    static final int KME_MODE_EXACT = 0, KME_MODE_FUNDED = 1;
    static final int KME_FLAG_EXACT_LEDGER = 1, KME_FLAG_SERIAL_FALLBACK = 2;
    static final int KME_OK = 0;
    static final int ROW_BYTES = 48;    // kme_row: oid, aid, sid, prev (long); action, price, size (int); kind, has_prev
    public static final String COMMIT_STORE = "MatchingEngineCommit";
    public static final String COMMIT_LOG = "MatchingEngineCommitLog";
    static final String COMMIT_KEY = "checkpoint";
    static final String CHUNK_PREFIX = "c:";                       // state chunks: "c:<index>:<hash>"
    static final int CHUNK_BYTES = 512 << 10;                      // below Kafka's default message size

    private static native long create(int mode, int maxSymbols, int maxEpoch, long maxResting, int maxTrades,
                                      int maxAccounts, int flags, int device, int nDevices, long ledgerCapacity);
    private static native void destroy(long h);
    private static native ByteBuffer buffer(long h, int slot, int column);
    private static native int submit(long h, int slot, int n);
    private static native int poll(long h);
    private static native int complete(long h, int slot, long[] status);
    private static native void forwarded(long h, int slot);
    private static native String statusText(int status);
    static native int checkpoint(long h, String path, long offset, long generation, long[] info);
    static native int restore(long h, String path, long[] out);
    static native int stateChunks(long h, String path, int chunkBytes, long[] hashes, long[] changed);
    static native int inspect(String path, long[] out);
    static native int shardStatus(long h, long[] out);

    private final int epoch;
    private final int maxTrades;
    private final int mode, flags, maxSymbols, maxAccounts, device, nDevices;
    private final long maxResting, ledgerCapacity;
    private ProcessorContext context;
    private long h;
    private File checkpointFile;
    private KeyValueStore<String, byte[]> commitLog;
    private long generation = 0;                    // of the last checkpoint written or restored
    private long[] chunkHashes = new long[0];        // the chunks the commit log's record names
    // per slot: the six Order columns (KP:451-456) and the MatchOut rows
    private final ByteBuffer[] action = new ByteBuffer[2], oid = new ByteBuffer[2], aid = new ByteBuffer[2],
            sid = new ByteBuffer[2], price = new ByteBuffer[2], size = new ByteBuffer[2], rows = new ByteBuffer[2];
    private final int[] count = new int[2];          // records buffered in the slot
    private final boolean[] busy = new boolean[2];   // in flight, or its rows not forwarded yet
    private int fill = 0;                            // the slot process() writes into
    private int oldest = 0;                          // the slot of the oldest epoch in flight
    private int inflight = 0;
    private final int[] ready = new int[2];          // completed slots whose rows wait to be forwarded, oldest first
    private int nReady = 0;
    private final int[] readyRows = new int[2];
    private final long[][] readyStatus = new long[2][4];
    private long lastOffset = -1;                    // Kafka offset of the last record taken into an epoch
    private long skipThrough = -1;                   // re-delivered records at or below it are in the checkpoint
    private long checkpointed = -1;                  // the offset the checkpoint on disk covers

    public GpuMatchingEngine() {
        // 65,537 symbol groups: sids up to 65,536 (BASELINE C3's universe is 1..65,536)
        // (ledger capacity: the initial size only -- Balances / Positions grow between epochs)
        this(1 << 16, 1 << 18, KME_MODE_FUNDED, KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK, 65537, 1 << 20,
             1L << 26, 0, 1, 1L << 20);
    }

    // nDevices > 1: the symbols keyed over GPUs device .. device + nDevices - 1 behind this one processor
    // (kme_multi: FUNDED shards; with the default flags an epoch no shard's funded bound can prove
    // consolidates the stream onto one exact engine on `device` -- the exact ledger couples every
    // symbol -- instead of failing; flags 0: such an epoch is fatal, KME_E_UNFUNDED)
    public GpuMatchingEngine(int epoch, int maxTrades, int mode, int flags, int maxSymbols, int maxAccounts,
                             long maxResting, int device, int nDevices, long ledgerCapacity) {
        this.epoch = epoch;
        this.maxTrades = maxTrades;
        this.mode = mode;
        this.flags = flags;
        this.maxSymbols = maxSymbols;
        this.maxAccounts = maxAccounts;
        this.maxResting = maxResting;
        this.device = device;
        this.nDevices = nDevices;
        this.ledgerCapacity = ledgerCapacity;
    }

    @Override
    public void init(ProcessorContext context) {                         // KP:86-93
        this.context = context;
        this.h = create(mode, maxSymbols, epoch, maxResting, maxTrades, maxAccounts, flags, device, nDevices,
                        ledgerCapacity);
        for (int s = 0; s < 2; s++) {
            action[s] = buffer(h, s, 0).order(ByteOrder.nativeOrder());
            oid[s] = buffer(h, s, 1).order(ByteOrder.nativeOrder());
            aid[s] = buffer(h, s, 2).order(ByteOrder.nativeOrder());
            sid[s] = buffer(h, s, 3).order(ByteOrder.nativeOrder());
            price[s] = buffer(h, s, 4).order(ByteOrder.nativeOrder());
            size[s] = buffer(h, s, 5).order(ByteOrder.nativeOrder());
            rows[s] = buffer(h, s, 6).order(ByteOrder.nativeOrder());
        }
        final StateStore hook = context.getStateStore(COMMIT_STORE);
        if (hook instanceof CommitHook) ((CommitHook) hook).owner = this;
        @SuppressWarnings("unchecked")
        final KeyValueStore<String, byte[]> log = (KeyValueStore<String, byte[]>) context.getStateStore(COMMIT_LOG);
        commitLog = log;
        checkpointFile = new File(context.stateDir(), "kme-" + context.taskId() + ".ckpt");
        final byte[] committed = commitLog.get(COMMIT_KEY);           // restored from the changelog
        // generation, offset, bytes, digest, chunk bytes, chunk count, the chunks' hashes
        final ByteBuffer want = committed == null ? null : ByteBuffer.wrap(committed);
        if (want != null) {
            chunkHashes = new long[(int) want.getLong(40)];
            for (int k = 0; k < chunkHashes.length; k++) chunkHashes[k] = want.getLong(48 + 8 * k);
            if (!isCommitted(checkpointFile, want)) rebuildFromLog(want);  // the task moved, or an older file
        }
        if (checkpointFile.exists()) {                                  // the state of the last commit
            final long[] r = new long[9];
            final int rc = restore(h, checkpointFile.getPath(), r);
            if (rc != KME_OK) throw new IllegalStateException("kme restore: " + statusText(rc));
            if (want != null && (r[6] < want.getLong(0) ||
                                 (r[6] == want.getLong(0) && (r[7] != want.getLong(16) || r[8] != want.getLong(24)))))
                throw new IllegalStateException("kme: " + checkpointFile + " (generation " + r[6] + ") is not the committed "
                                                + "checkpoint (generation " + want.getLong(0) + ", offset " + want.getLong(8) + ")");
            generation = r[6];
            skipThrough = checkpointed = lastOffset = r[0];
            if (want != null && isCommitted(checkpointFile, want)) {      // the chunks the changelog holds
                final long[] hs = new long[(int) ((r[7] + CHUNK_BYTES - 1) / CHUNK_BYTES)], ch = new long[1 + hs.length];
                stateChunks(h, checkpointFile.getPath(), CHUNK_BYTES, hs, ch);
            }
            for (int k = 0; k < (int) r[1]; k++) {                      // rows not forwarded before the crash
                final int s = (int) r[2 + 2 * k];
                readyRows[s] = (int) r[3 + 2 * k];
                readyStatus[s][0] = KME_OK;
                busy[s] = true;
                ready[nReady++] = s;
            }
        } else if (want != null) {                                      // committed state, not rebuilt
            throw new IllegalStateException("kme: the commit log names checkpoint generation " + want.getLong(0) + " (offset "
                                            + want.getLong(8) + ") but neither " + checkpointFile + " nor the changelogged "
                                            + "chunks hold it: the book cannot be rebuilt");
        }
        context.schedule(Duration.ofMillis(1), PunctuationType.WALL_CLOCK_TIME, ts -> punctuate());
    }

    @Override
    public void process(String key, Order o) {                          // KP:96
        forwardReady();
        final long offset = context.offset();
        if (offset <= skipThrough) return;                              // taken before the restored checkpoint
        while (busy[fill]) {                                            // both slots busy
            if (nReady > 0) forwardReady();
            else completeOldest(true);
        }
        final int n = count[fill];
        action[fill].putInt(4 * n, o.action);
        oid[fill].putLong(8 * n, o.oid);
        aid[fill].putLong(8 * n, o.aid);
        sid[fill].putLong(8 * n, o.sid);
        price[fill].putInt(4 * n, o.price);
        size[fill].putInt(4 * n, o.size);
        count[fill] = n + 1;
        lastOffset = offset;
        if (count[fill] == epoch) flush();
    }

    // Sends the slot being filled as one epoch (asynchronous: returns once it is queued).
    private void flush() {
        if (count[fill] == 0) return;
        while (inflight == 2) completeOldest(true);
        final int rc = submit(h, fill, count[fill]);
        if (rc != KME_OK) throw new IllegalStateException("kme submit: " + statusText(rc));
        if (inflight == 0) oldest = fill;
        busy[fill] = true;
        inflight++;
        fill ^= 1;
    }

    // Waits for the oldest epoch in flight; its rows become ready, and are forwarded now unless the
    // caller is the commit point.
    private void completeOldest(boolean forward) {
        final int s = oldest;
        readyRows[s] = complete(h, s, readyStatus[s]);
        ready[nReady++] = s;
        inflight--;
        oldest = s ^ 1;
        if (forward) forwardReady();
    }

    // Forwards the ready rows, oldest epoch first, in the reference's order (IN, fills, OUT per record).
    private void forwardReady() {
        while (nReady > 0) {
            final int s = ready[0];
            final ByteBuffer r = rows[s];
            for (int k = 0; k < readyRows[s]; k++) {
                final int b = ROW_BYTES * k;
                final Order o = new Order(r.getInt(b + 32), r.getLong(b), r.getLong(b + 8), r.getLong(b + 16),
                                          r.getInt(b + 36), r.getInt(b + 40));
                final int kind = r.get(b + 44);
                if (kind == 2 && r.get(b + 45) != 0) o.prev = r.getLong(b + 24);     // OUT echo of an append (KP:217)
                context.forward(kind == 0 ? "IN" : "OUT", o);
            }
            forwarded(h, s);
            ready[0] = ready[1];
            nReady--;
            busy[s] = false;
            count[s] = 0;
            if (readyStatus[s][0] != KME_OK)                            // the stream thread dies
                throw new IllegalStateException(statusText((int) readyStatus[s][0]));
        }
    }

    // Wall-clock punctuation: forward every epoch the GPU has finished, without blocking, and send
    // a partly filled epoch when a slot is free.
    private void punctuate() {
        forwardReady();
        while (inflight > 0) {
            final int p = poll(h);
            if (p < 0) throw new IllegalStateException("kme poll: " + statusText(-p));
            if (p == 0) break;
            completeOldest(true);
        }
        if (inflight < 2 && count[fill] > 0 && !busy[fill]) flush();
    }

    // The commit point: the commit hook's flush(), before Kafka Streams commits the offsets of every
    // record process() took.  Nothing is forwarded here; the checkpoint keeps what is not forwarded.
    void commitPoint() {
        if (h == 0 || lastOffset == checkpointed) return;               // nothing taken since the last one
        flush();
        while (inflight > 0) completeOldest(false);
        for (int k = 0; k < nReady; k++)                                // a faulted epoch is not a commit point
            if (readyStatus[ready[k]][0] != KME_OK) throw new IllegalStateException(statusText((int) readyStatus[ready[k]][0]));
        final long[] info = new long[2];                              // the file's size and digest
        final int rc = checkpoint(h, checkpointFile.getPath(), lastOffset, generation + 1, info);
        if (rc != KME_OK) throw new IllegalStateException("kme checkpoint: " + statusText(rc));
        generation += 1;
        // the state changelog: the chunks whose content changed, under keys no earlier record names ...
        final long[] hashes = new long[(int) ((info[0] + CHUNK_BYTES - 1) / CHUNK_BYTES)], changed = new long[1 + hashes.length];
        final int n = stateChunks(h, checkpointFile.getPath(), CHUNK_BYTES, hashes, changed);
        if (n < 0) throw new IllegalStateException("kme state chunks: " + statusText(-n));
        try (RandomAccessFile f = new RandomAccessFile(checkpointFile, "r")) {
            for (int k = 0; k < (int) changed[0]; k++) {
                final int c = (int) changed[1 + k];
                final byte[] b = new byte[(int) Math.min(CHUNK_BYTES, info[0] - (long) c * CHUNK_BYTES)];
                f.seek((long) c * CHUNK_BYTES);
                f.readFully(b);
                commitLog.put(chunkKey(c, hashes[c]), b);
            }
        } catch (IOException e) {
            throw new UncheckedIOException(e);
        }
        // ... then the record that names them, before Kafka Streams commits the offsets
        final ByteBuffer rec = ByteBuffer.allocate(48 + 8 * n).putLong(generation).putLong(lastOffset).putLong(info[0])
                                         .putLong(info[1]).putLong(CHUNK_BYTES).putLong(n);
        for (int k = 0; k < n; k++) rec.putLong(hashes[k]);
        commitLog.put(COMMIT_KEY, rec.array());
        // chunks the record no longer names (their keys were the previous record's)
        for (int k = 0; k < chunkHashes.length; k++)
            if (k >= n || chunkHashes[k] != hashes[k]) commitLog.delete(chunkKey(k, chunkHashes[k]));
        chunkHashes = java.util.Arrays.copyOf(hashes, n);
        checkpointed = lastOffset;
    }

    static String chunkKey(int index, long hash) { return CHUNK_PREFIX + index + ":" + Long.toHexString(hash); }

    // the file at f is the one the record names (its trailer: size and digest)
    private static boolean isCommitted(File f, ByteBuffer want) {
        if (!f.exists()) return false;
        final long[] t = new long[3];
        return inspect(f.getPath(), t) == KME_OK && t[0] == want.getLong(16) && t[2] == want.getLong(24);
    }

    // The committed checkpoint rebuilt from the changelogged chunks into the state directory (written
    // beside it, then renamed over it); left as it is when a chunk is missing or the result is not the
    // committed file (init() then takes a newer local file, or refuses).
    private void rebuildFromLog(ByteBuffer want) {
        if (want.getLong(32) != CHUNK_BYTES) return;
        final File tmp = new File(checkpointFile.getPath() + ".log");
        try (FileOutputStream out = new FileOutputStream(tmp)) {
            for (int k = 0; k < chunkHashes.length; k++) {
                final byte[] b = commitLog.get(chunkKey(k, chunkHashes[k]));
                if (b == null) return;
                out.write(b);
            }
            out.getFD().sync();
        } catch (IOException e) {
            throw new UncheckedIOException(e);
        }
        if (!isCommitted(tmp, want)) return;
        try {
            Files.move(tmp.toPath(), checkpointFile.toPath(), StandardCopyOption.REPLACE_EXISTING, StandardCopyOption.ATOMIC_MOVE);
        } catch (IOException e) {
            throw new UncheckedIOException(e);
        }
    }

    // nDevices > 1: {engines, consolidated, can consolidate, failed, history records, history cap,
    // history records made durable, checkpoint generation} -- whether an epoch no shard can prove is
    // survivable now (kme_multi_info); null for one engine
    public long[] shardStatus() {
        final long[] out = new long[8];
        return shardStatus(h, out) == KME_OK ? out : null;
    }

    @Override
    public void close() {                                               // KP:129
        try {
            forwardReady();
            flush();
            while (inflight > 0) completeOldest(true);
            commitPoint();                                              // everything forwarded: the final state
        } finally {
            destroy(h);
            h = 0;
        }
    }

    // ---- the commit hook: a state store whose flush() is the processor's commit point
    public static StoreBuilder<CommitHook> commitHook() {
        return new CommitHookBuilder(COMMIT_STORE);
    }

    // ---- the commit log: which checkpoint each commit point wrote, changelogged (logging is on by
    // default for a persistent key-value store; caching off, so the put reaches the changelog producer
    // inside the commit, before the offsets)
    public static StoreBuilder<KeyValueStore<String, byte[]>> commitLog() {
        return Stores.keyValueStoreBuilder(Stores.persistentKeyValueStore(COMMIT_LOG), Serdes.String(), Serdes.ByteArray())
                     .withCachingDisabled();
    }

    public static final class CommitHook implements StateStore {
        private final String name;
        private GpuMatchingEngine owner;
        private boolean open;

        CommitHook(String name) { this.name = name; }

        @Override
        public String name() { return name; }

        @Override
        public void init(ProcessorContext context, StateStore root) {
            context.register(root, (key, value) -> { });              // holds nothing (the commit log does)
            open = true;
        }

        @Override
        public void flush() {                                          // before the offsets are committed
            if (owner != null) owner.commitPoint();
        }

        @Override
        public void close() { open = false; }

        @Override
        public boolean persistent() { return false; }

        @Override
        public boolean isOpen() { return open; }
    }

    static final class CommitHookBuilder implements StoreBuilder<CommitHook> {
        private final String name;

        CommitHookBuilder(String name) { this.name = name; }

        public StoreBuilder<CommitHook> withCachingEnabled() { return this; }

        public StoreBuilder<CommitHook> withCachingDisabled() { return this; }

        public StoreBuilder<CommitHook> withLoggingEnabled(Map<String, String> config) { return this; }

        public StoreBuilder<CommitHook> withLoggingDisabled() { return this; }

        public CommitHook build() { return new CommitHook(name); }

        public Map<String, String> logConfig() { return Collections.emptyMap(); }

        public boolean loggingEnabled() { return false; }

        public String name() { return name; }
    }
}
