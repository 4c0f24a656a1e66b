"""JUnit XML reports for test runs.

Parity: /root/reference/py/test_util.py:8-60 (TestCase + create_junit_xml_file). Written with
xml.etree instead of string templates so names/messages are escaped; a GCS upload is out of scope (no cloud
SDK): the path is always local.
"""
from __future__ import annotations

import os
import time
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class TestCase:
    class_name: str = ""
    name: str = ""
    time: float = 0.0  # seconds
    failure: Optional[str] = None


def junit_xml(cases: List[TestCase]) -> str:
    failures = sum(1 for c in cases if c.failure)
    total = sum(c.time for c in cases)
    suite = ET.Element("testsuite", failures=str(failures), tests=str(len(cases)), time="%g" % total)
    for c in cases:
        e = ET.SubElement(suite, "testcase", classname=c.class_name, name=c.name, time="%g" % c.time)
        if c.failure:
            ET.SubElement(e, "failure").text = c.failure
    return ET.tostring(suite, encoding="unicode")


def create_junit_xml_file(cases: List[TestCase], output_path: str) -> str:
    d = os.path.dirname(output_path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(output_path, "w") as f:
        f.write(junit_xml(cases))
    return output_path


class Timer:
    def __enter__(self):
        self.t0 = time.time()
        return self

    def __exit__(self, *a):
        self.elapsed = time.time() - self.t0
