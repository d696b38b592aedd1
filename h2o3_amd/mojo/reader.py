"""Inspect a MOJO (reference: hex/genmodel/tools/PrintMojo)."""
import json
import zipfile


def describe(path):
    with zipfile.ZipFile(path) as z:
        return {"ini": z.read("model.ini").decode(), "meta": json.loads(z.read("model.json")),
                "files": z.namelist()}
