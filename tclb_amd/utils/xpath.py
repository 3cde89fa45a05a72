"""CLI XPath editing of the case XML (reference: src/xpath_modification.cpp:4-163).

Operators: ``XPATH = value`` (XPATH ends with /@attr), ``XPATH @attr = value``
(add/change attribute), ``XPATH insert|inject [first|last|after|before] '<xml/>'``,
``XPATH delete``, ``XPATH print``, ``-s file`` (save), ``-x`` (exit).  XPath subset of
xml.etree (child paths, ``//``, ``[@a='v']`` predicates, indices)."""
from __future__ import annotations

import xml.etree.ElementTree as ET
from typing import List, Tuple

from .log import log


class XPathError(ValueError):
    pass


def _split_attr(path: str):
    if "/@" in path:
        p, a = path.rsplit("/@", 1)
        return p, a
    if path.startswith("@"):
        return ".", path[1:]
    return path, None


def _select(root: ET.Element, path: str) -> List[ET.Element]:
    p = path.strip()
    if p.startswith("/" + root.tag):
        p = "." + p[len(root.tag) + 1:]
    elif p.startswith("//"):
        p = "." + p
    elif p.startswith("/"):
        p = "." + p
    if p in (".", ""):
        return [root]
    return root.findall(p)


def _parents(root):
    return {c: p for p in root.iter() for c in p}


def apply_edits(root: ET.Element, argv: List[str]) -> Tuple[ET.Element, bool]:
    i = 0
    n = len(argv)
    while i < n:
        a = argv[i]
        if a == "-s":
            i += 1
            if i >= n:
                raise XPathError("no filename for -s")
            ET.ElementTree(root).write(argv[i])
            i += 1
            continue
        if a == "-x":
            log.output("Gracefully exiting")
            return root, True
        path, attr = _split_attr(a)
        found = _select(root, path)
        i += 1
        if i >= n:
            raise XPathError("no operator in xpath evaluation")
        add_attr = None
        if argv[i].startswith("@"):
            add_attr = argv[i][1:]
            i += 1
        op = argv[i]
        if op == "=":
            i += 1
            if i >= n:
                raise XPathError("XPATH: No value supplied to = operator")
            if not found:
                raise XPathError("XPATH: Nothing selected for substitution")
            for e in found:
                name = add_attr or attr
                if name is None:
                    raise XPathError("XPATH: Operator = can only be used for attributes")
                if add_attr is None and e.get(name) is None:
                    raise XPathError(f"XPATH: attribute {name} not present (use 'PATH @{name} = v' to add)")
                e.set(name, argv[i])
                log.output(f"XPATH: Set attr {name} to \"{argv[i]}\" in <{e.tag} />")
            i += 1
        elif op in ("inject", "insert"):
            i += 1
            where = "last"
            if i < n and argv[i] in ("last", "first", "after", "before"):
                where = argv[i]
                i += 1
            if i >= n:
                raise XPathError("XPATH: No value supplied to inject operator")
            new = ET.fromstring(argv[i])
            if not found:
                raise XPathError("XPATH: Nothing selected for injection")
            e = found[0]
            par = _parents(root)
            if where == "last":
                e.append(new)
            elif where == "first":
                e.insert(0, new)
            else:
                p = par.get(e)
                if p is None:
                    raise XPathError("cannot insert next to the root")
                k = list(p).index(e)
                p.insert(k + 1 if where == "after" else k, new)
            i += 1
        elif op == "delete":
            par = _parents(root)
            for e in found:
                if attr is not None:
                    e.attrib.pop(attr, None)
                else:
                    par[e].remove(e)
            i += 1
        elif op == "print":
            for e in found:
                if attr is not None:
                    log.output(f"XPATH: Attr: {attr}=\"{e.get(attr)}\"")
                else:
                    log.output(f"XPATH: Node: {e.tag}")
            i += 1
        else:
            raise XPathError(f"Unknown operator in xpath evaluation: {op}")
    return root, False


def strip_comments(root: ET.Element) -> ET.Element:
    return root  # ElementTree drops comments by default


def rewrite_deprecated_params(root):
    """<Params a="1" b-zone="2" gauge="g"/> -> one <Param name= value= [zone=] [gauge=]/>
    per attribute, in place, and switch the config to permissive mode (reference
    src/main.cpp:261-293).  Returns the number of rewritten elements."""
    count = 0
    for parent in list(root.iter()):
        kids = list(parent)
        for node in kids:
            if node.tag != "Params":
                continue
            count += 1
            gauge = node.get("gauge")
            pos = list(parent).index(node)
            new = []
            for k, v in node.attrib.items():
                if k == "gauge":
                    continue
                par, _, zone = k.partition("-")
                p = ET.Element("Param", {"name": par, "value": v})
                if zone:
                    p.set("zone", zone)
                if gauge is not None:
                    p.set("gauge", gauge)
                p.tail = node.tail
                new.append(p)
            parent.remove(node)
            for j, p in enumerate(new):
                parent.insert(pos + j, p)
    if count:
        root.set("permissive", "true")
    return count


def load_case(path: str) -> ET.Element:
    """Parse a case file the way pugixml accepts it (reference src/main.cpp:238-262):
    comments or blank text before the ``<?xml ...?>`` declaration are dropped (several
    reference cases start with ``<!-- To be used with <model> -->``), and a byte-order
    mark is ignored."""
    with open(path, "rb") as f:
        raw = f.read()
    text = raw.decode("utf-8-sig", errors="replace")
    k = text.find("<?xml")
    if k > 0:
        head = text[:k]
        # only comments / whitespace may precede the declaration
        import re
        if re.sub(r"<!--.*?-->", "", head, flags=re.S).strip() == "":
            text = text[k:]
    try:
        return ET.fromstring(text)
    except ET.ParseError as e:
        raise XPathError(f"cannot parse case file {path}: {e}") from None
