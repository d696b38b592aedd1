"""Inspect a MOJO (reference: hex/genmodel/tools/PrintMojo)."""
import json
import zipfile


def describe(path):
    """model.ini text, metadata and file list of a MOJO in either layout
    (this platform's model.json, or the reference's model.ini-only layout)."""
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        ini = z.read("model.ini").decode()
        if "model.json" in names:
            meta = json.loads(z.read("model.json"))
        else:
            from .h2o_mojo import H2OMojoModel
            meta = H2OMojoModel(path).meta
        return {"ini": ini, "meta": meta, "files": names}
