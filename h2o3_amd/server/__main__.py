"""`python -m h2o3_amd.server [--ip IP] [--port PORT]`: serve the /3 REST API
(the reference's `java -jar h2o.jar` entry point, water/H2OApp.java), so the
reference clients (h2o-py `h2o.connect(url=...)`, h2o-r `h2o.init(ip, port,
startH2O = FALSE)`) can drive this process and its GPU."""
import argparse

from .rest import start


def main():
    import faulthandler
    import signal
    # `kill -USR1 <pid>` dumps every thread's stack (diagnosing a stuck rank)
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    ap = argparse.ArgumentParser(prog="python -m h2o3_amd.server")
    ap.add_argument("--ip", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=54321)
    ap.add_argument("--log-level", default="warning")
    ap.add_argument("--hash-login", action="store_true", help="HTTP Basic auth against --login-conf (Jetty realm file)")
    ap.add_argument("--login-conf", default=None, help="realm file: 'user: password[,role]' (plain, MD5:, OBF:)")
    ap.add_argument("--ssl-certfile", default=None, help="PEM certificate: serve HTTPS")
    ap.add_argument("--ssl-keyfile", default=None, help="PEM private key for --ssl-certfile")
    ap.add_argument("--flow-dir", default=None, help="NodePersistentStorage directory for saved Flow notebooks "
                                                     "(default $H2O3_FLOW_DIR or ~/h2oflows)")
    a = ap.parse_args()
    if a.hash_login and not a.login_conf:
        ap.error("--hash-login needs --login-conf")
    start(ip=a.ip, port=a.port, log_level=a.log_level, login_conf=a.login_conf if a.hash_login else None,
          ssl_certfile=a.ssl_certfile, ssl_keyfile=a.ssl_keyfile, flow_dir=a.flow_dir)


if __name__ == "__main__":
    main()
