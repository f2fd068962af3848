// CurveClientMechanism with its MESSAGE phase on the MI355X: the handshake, metadata and ZAP flow
// are the reference's own (inherited), and once status() == READY every encode / decode runs on
// the device through GpuCurveMessageBatch (CurveClientMechanism.java:126-224), one message at a time as
// StreamEngine calls it (:1052-1098), or many at once through encodeBatch / decodeBatch for a
// caller that collects them (Mechanism.java:202-210; SURVEY.md section 7 step 6).
// Plugged in by Mechanisms.CURVE.create (zmq/io/mechanism/Mechanisms.java:80-89):
//     return new GpuCurveClientMechanism(session, options);
package zmq.io.mechanism.curve;

import java.util.Collections;
import java.util.List;

import zmq.Msg;
import zmq.Options;
import zmq.io.SessionBase;

public class GpuCurveClientMechanism extends CurveClientMechanism implements AutoCloseable
{
    private final Options         opts;
    private GpuCurveMessageBatch batch;   // created at the first MESSAGE, after the handshake

    public GpuCurveClientMechanism(SessionBase session, Options options)
    {
        super(session, options);
        this.opts = options;
    }

    private GpuCurveMessageBatch batch()
    {
        if (batch == null) {
            assert (status() == Status.READY);
            batch = new GpuCurveMessageBatch(this, CurveClientMechanism.class, false, session, opts.errno);
        }
        return batch;
    }

    @Override
    public Msg encode(Msg msg)
    {
        return batch().encode(Collections.singletonList(msg)).get(0);
    }

    // null on a failed frame, with the reference's event raised and errno = EPROTO
    @Override
    public Msg decode(Msg msg)
    {
        List<Msg> out = batch().decode(Collections.singletonList(msg));
        return out.isEmpty() ? null : out.get(0);
    }

    // every message sealed in one device batch, in order, cnNonce advanced by msgs.size()
    public List<Msg> encodeBatch(List<Msg> msgs)
    {
        return batch().encode(msgs);
    }

    // the decoded prefix up to the first failing body; lastBatchFailed() then says the connection
    // must be torn down (the event was raised, as decode returning null)
    public List<Msg> decodeBatch(List<Msg> bodies)
    {
        return batch().decode(bodies);
    }

    public boolean lastBatchFailed()
    {
        return batch != null && batch.failed();
    }

    @Override
    public void close()
    {
        if (batch != null) {
            batch.close();
            batch = null;
        }
    }
}
