"""In-process broker semantics: held messages only for never-subscribed topics, bounded, forgotten when a run ends,
and replayed ahead of any later publish."""
import threading

from fedml_amd.core.distributed.communication.pubsub import InProcessBroker


def test_hold_only_until_first_subscriber_then_drop():
    b = InProcessBroker(max_held=3)
    for i in range(5):
        b.publish("t", bytes([i]))
    got = []
    cb = lambda t, p: got.append(p[0])   # noqa: E731
    b.subscribe("t", cb)
    assert got == [2, 3, 4]                      # capped: the oldest two were dropped
    b.unsubscribe_all(cb)
    b.publish("t", b"\x09")                      # the topic has had a subscriber: not held for the next one
    got2 = []
    b.subscribe("t", lambda t, p: got2.append(p[0]))
    assert got2 == [] and b.dropped == 3


def test_forget_drops_a_finished_runs_held_messages():
    b = InProcessBroker()
    b.publish("fedml_7_0_1", b"late")
    b.publish("fedml_8_0_1", b"keep")
    b.forget("fedml_7_")
    a, c = [], []
    b.subscribe("fedml_7_0_1", lambda t, p: a.append(p))
    b.subscribe("fedml_8_0_1", lambda t, p: c.append(p))
    assert a == [] and c == [b"keep"]


def test_held_replay_precedes_concurrent_publish():
    b = InProcessBroker()
    for i in range(200):
        b.publish("q", i.to_bytes(2, "little"))
    out = []
    started = threading.Event()

    def cb(t, p):
        started.set()
        out.append(int.from_bytes(p, "little"))

    def publisher():
        started.wait()
        for i in range(200, 260):
            b.publish("q", i.to_bytes(2, "little"))

    th = threading.Thread(target=publisher)
    th.start()
    b.subscribe("q", cb)
    th.join()
    assert out == list(range(260))
