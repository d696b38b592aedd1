import sys

PY2 = False
PY3 = True


def with_metaclass(meta, *bases):
    """Class with metaclass `meta` deriving from `bases` (Py3 form)."""
    class _Meta(meta):
        def __new__(cls, name, this_bases, d):
            return meta(name, bases, d)
    return type.__new__(_Meta, "temporary_class", (), {})


def viewitems(d):
    return d.items()


def viewkeys(d):
    return d.keys()


def viewvalues(d):
    return d.values()


native_str = str
string_types = (str,)
text_type = str
PYPY = "__pypy__" in sys.builtin_module_names
