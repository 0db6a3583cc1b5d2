"""MLOps runtime-log upload (reference ``core/mlops/mlops_runtime_log.py:122-194``): new log lines go to a
configured ``log_server_url`` as the reference's JSON request; the sent-line index persists, a failed POST
keeps the lines for the next attempt. The server here is a local ``http.server`` (air-gapped)."""
import json
import logging
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

from fedml_amd.arguments import Arguments
from fedml_amd.core.mlops.mlops_runtime_log import LogUploader, MLOpsRuntimeLog


def _server(status):
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            n = int(self.headers["Content-Length"])
            got.append(json.loads(self.rfile.read(n)))
            self.send_response(status[0])
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            self.wfile.write(b'{"code": "SUCCESS"}')

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, got


def test_uploader_sends_new_lines_resumes_and_retries(tmp_path):
    status = [500]
    srv, got = _server(status)
    url = f"http://127.0.0.1:{srv.server_port}/fedmlOpsServer/logs/update"
    log = tmp_path / "run.log"
    log.write_text("a\nb\n")
    up = LogUploader(str(log), url, run_id="7", edge_id=3, interval_s=60)
    assert up.upload_once() == 0 and up.failed_batches == 1          # server error: lines kept
    status[0] = 200
    assert up.upload_once() == 2
    assert got[-1]["logs"] == ["a\n", "b\n"] and got[-1]["run_id"] == "7" and got[-1]["edge_id"] == 3
    with open(log, "a") as f:
        f.write("c\n")
    up2 = LogUploader(str(log), url, run_id="7", edge_id=3)           # a restarted process resumes
    assert up2.upload_once() == 1 and got[-1]["logs"] == ["c\n"]
    assert up2.upload_once() == 0                                     # nothing new
    srv.shutdown()
    dead = LogUploader(str(log), "http://127.0.0.1:9/none", run_id="7", edge_id=3, timeout_s=1)
    dead.line_index = 0
    assert dead.upload_once() == 0                                    # unreachable: no exception


def test_runtime_log_uploads_records(tmp_path):
    srv, got = _server([200])
    args = Arguments.from_dict({"x": {"rank": 1, "run_id": "r1", "log_file_dir": str(tmp_path), "log_to_file": True,
                                      "log_server_url": f"http://127.0.0.1:{srv.server_port}/logs",
                                      "log_upload_interval_s": 30}})
    rl = MLOpsRuntimeLog(args).init_logs()
    assert rl.uploader is not None
    logging.info("round 0 done")
    rl.close()
    lines = [ln for req in got for ln in req["logs"]]
    assert any("round 0 done" in ln and "[FedML-Client(1)" in ln for ln in lines)
    srv.shutdown()
    for h in list(logging.getLogger().handlers):
        logging.getLogger().removeHandler(h)
