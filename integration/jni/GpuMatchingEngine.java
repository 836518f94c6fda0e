// GpuMatchingEngine -- the MI355X matching engine behind the reference's Processor interface, the
// one-line swap at the topology (KProcessor.java:52):
//
//     .addProcessor("MatchingEngine", GpuMatchingEngine::new, "Source")
//
// Like the reference's MatchingEngine (KP:63) it is a Processor<String, Order> over the reference's
// own top-level Order class (KP:449-475), in the same (default) package; it uses only Order's public
// fields and its six-argument creator (KP:463-465).  tests/test_java_processor.py holds this file to
// KProcessor.java's declarations.
//
// Contract kept from MatchingEngine.process (KP:96-126): for every input record the processor
// forwards ("IN", order), then the maker and the taker fill of each trade (keyed "OUT", KP:272-273),
// then ("OUT", order) -- same order, same field values.  The difference is timing: records are
// buffered into an epoch and forwarded when the epoch completes; the offset commit is requested after
// the epoch's records are forwarded, never before.
//
// Path at rate (include/kme.h, "Host epochs at device rate"): two slots of JVM direct ByteBuffers
// hold an epoch's Order columns (native byte order) and the MatchOut rows that come back; the native
// side registers them once, so an epoch crosses PCIe straight from and to them.  While the GPU runs
// epoch k, process() fills the other slot; the wall-clock punctuator polls (never blocks) and
// forwards a finished epoch, and sends a partly filled one so that latency stays bounded.
//
// Faults: the records before a fault took effect and are forwarded and committed (as the reference's
// per-record commit would have, KP:97, 124-125); then the processor fails like the reference's
// stream thread.  The default flags (EXACT_LEDGER | SERIAL_FALLBACK) give the reference's result for
// any stream, so KME_E_UNFUNDED cannot occur; in a configuration without SERIAL_FALLBACK it is fatal
// here too (its records were not processed, and a processor cannot hand records back to Kafka).
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.time.Duration;

import org.apache.kafka.streams.processor.Processor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.PunctuationType;

public final class GpuMatchingEngine implements Processor<String, Order> {
    static { System.loadLibrary("kme_jni"); }

    // include/kme.h
    static final int KME_MODE_EXACT = 0, KME_MODE_FUNDED = 1;
    static final int KME_FLAG_EXACT_LEDGER = 1, KME_FLAG_SERIAL_FALLBACK = 2;
    static final int KME_OK = 0;
    static final int ROW_BYTES = 48;    // kme_row: oid, aid, sid, prev (long); action, price, size (int); kind, has_prev

    private static native long create(int mode, int maxSymbols, int maxEpoch, long maxResting, int maxTrades,
                                      int maxAccounts, int flags, int device);
    private static native void destroy(long h);
    private static native int bind(long h, int slot, ByteBuffer action, ByteBuffer oid, ByteBuffer aid, ByteBuffer sid,
                                   ByteBuffer price, ByteBuffer size, ByteBuffer rows);
    private static native int submit(long h, int slot, int n);
    private static native int poll(long h);
    private static native int complete(long h, int slot, long[] status);
    private static native String statusText(int status);
    static native int checkpoint(long h, String path);
    static native int restore(long h, String path);

    private final int epoch;
    private final int maxTrades;
    private final int mode, flags, maxSymbols, maxAccounts, device;
    private final long maxResting;
    private ProcessorContext context;
    private long h;
    // per slot: the six Order columns (KP:451-456) and the MatchOut rows
    private final ByteBuffer[] action = new ByteBuffer[2], oid = new ByteBuffer[2], aid = new ByteBuffer[2],
            sid = new ByteBuffer[2], price = new ByteBuffer[2], size = new ByteBuffer[2], rows = new ByteBuffer[2];
    private final int[] count = new int[2];          // records buffered in the slot
    private final boolean[] busy = new boolean[2];   // the slot's epoch is in flight
    private int fill = 0;                            // the slot process() writes into
    private int oldest = 0;                          // the slot of the oldest epoch in flight
    private int inflight = 0;
    private final long[] status = new long[4];

    public GpuMatchingEngine() {
        this(1 << 16, 1 << 18, KME_MODE_FUNDED, KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK, 1 << 16, 1 << 20,
             1L << 26, 0);
    }

    public GpuMatchingEngine(int epoch, int maxTrades, int mode, int flags, int maxSymbols, int maxAccounts,
                             long maxResting, int device) {
        this.epoch = epoch;
        this.maxTrades = maxTrades;
        this.mode = mode;
        this.flags = flags;
        this.maxSymbols = maxSymbols;
        this.maxAccounts = maxAccounts;
        this.maxResting = maxResting;
        this.device = device;
        for (int s = 0; s < 2; s++) {
            action[s] = direct(4L * epoch);
            oid[s] = direct(8L * epoch);
            aid[s] = direct(8L * epoch);
            sid[s] = direct(8L * epoch);
            price[s] = direct(4L * epoch);
            size[s] = direct(4L * epoch);
            rows[s] = direct((long) ROW_BYTES * (2L * epoch + 2L * maxTrades));
        }
    }

    private static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE) throw new IllegalArgumentException("kme: buffer over 2 GiB");
        return ByteBuffer.allocateDirect((int) bytes).order(ByteOrder.nativeOrder());
    }

    @Override
    public void init(ProcessorContext context) {                         // KP:86-93
        this.context = context;
        this.h = create(mode, maxSymbols, epoch, maxResting, maxTrades, maxAccounts, flags, device);
        for (int s = 0; s < 2; s++) {
            final int rc = bind(h, s, action[s], oid[s], aid[s], sid[s], price[s], size[s], rows[s]);
            if (rc != KME_OK) throw new IllegalStateException("kme bind: " + statusText(rc));
        }
        context.schedule(Duration.ofMillis(1), PunctuationType.WALL_CLOCK_TIME, ts -> punctuate());
    }

    @Override
    public void process(String key, Order o) {                          // KP:96
        while (busy[fill]) completeOldest();                            // both slots in flight
        final int n = count[fill];
        action[fill].putInt(4 * n, o.action);
        oid[fill].putLong(8 * n, o.oid);
        aid[fill].putLong(8 * n, o.aid);
        sid[fill].putLong(8 * n, o.sid);
        price[fill].putInt(4 * n, o.price);
        size[fill].putInt(4 * n, o.size);
        count[fill] = n + 1;
        if (count[fill] == epoch) flush();
    }

    // Sends the slot being filled as one epoch (asynchronous: returns once it is queued).
    private void flush() {
        if (count[fill] == 0) return;
        while (inflight == 2) completeOldest();
        final int rc = submit(h, fill, count[fill]);
        if (rc != KME_OK) throw new IllegalStateException("kme submit: " + statusText(rc));
        if (inflight == 0) oldest = fill;
        busy[fill] = true;
        inflight++;
        fill ^= 1;
    }

    // Waits for the oldest epoch in flight, forwards its MatchOut rows in the reference's order and
    // commits them.
    private void completeOldest() {
        final int s = oldest;
        final int n = complete(h, s, status);
        final ByteBuffer r = rows[s];
        for (int k = 0; k < n; k++) {
            final int b = ROW_BYTES * k;
            final Order o = new Order(r.getInt(b + 32), r.getLong(b), r.getLong(b + 8), r.getLong(b + 16),
                                      r.getInt(b + 36), r.getInt(b + 40));
            final int kind = r.get(b + 44);
            if (kind == 2 && r.get(b + 45) != 0) o.prev = r.getLong(b + 24);     // OUT echo of an append (KP:217)
            context.forward(kind == 0 ? "IN" : "OUT", o);
        }
        busy[s] = false;
        count[s] = 0;
        inflight--;
        oldest = s ^ 1;
        context.commit();                                               // KP:125, once per epoch
        if (status[0] != KME_OK) throw new IllegalStateException(statusText((int) status[0]));   // the stream thread dies
    }

    // Wall-clock punctuation: forward every epoch the GPU has finished, without blocking, and send
    // a partly filled epoch when a slot is free.
    private void punctuate() {
        while (inflight > 0) {
            final int p = poll(h);
            if (p < 0) throw new IllegalStateException("kme poll: " + statusText(-p));
            if (p == 0) break;
            completeOldest();
        }
        if (inflight < 2 && count[fill] > 0) flush();
    }

    // Persistence in place of the RocksDB changelogs (KP:30-49): every epoch received so far is
    // completed first.
    public void checkpoint(String path) {
        flush();
        while (inflight > 0) completeOldest();
        final int rc = checkpoint(h, path);
        if (rc != KME_OK) throw new IllegalStateException("kme checkpoint: " + statusText(rc));
    }

    @Override
    public void close() {                                               // KP:129
        try {
            flush();
            while (inflight > 0) completeOldest();
        } finally {
            destroy(h);
            h = 0;
        }
    }
}
