"""`python -m h2o3_amd.server [--ip IP] [--port PORT]`: serve the /3 REST API
(the reference's `java -jar h2o.jar` entry point, water/H2OApp.java), so the
reference clients (h2o-py `h2o.connect(url=...)`, h2o-r `h2o.init(ip, port,
startH2O = FALSE)`) can drive this process and its GPU."""
import argparse

from .rest import start


def main():
    ap = argparse.ArgumentParser(prog="python -m h2o3_amd.server")
    ap.add_argument("--ip", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=54321)
    ap.add_argument("--log-level", default="warning")
    a = ap.parse_args()
    start(ip=a.ip, port=a.port, log_level=a.log_level)


if __name__ == "__main__":
    main()
