"""Kernel dispatch rows from a rocprofv3 kernel trace: the CSV (``--output-format csv``) or the
SQLite ``*_results.db`` it writes by default on this image, as dicts with the CSV's column names."""
from __future__ import annotations

import csv
import sqlite3

_MAP = {"name": "Kernel_Name", "start": "Start_Timestamp", "end": "End_Timestamp", "lds_size": "LDS_Block_Size",
        "vgpr_count": "VGPR_Count", "accum_vgpr_count": "Accum_VGPR_Count", "workgroup_x": "Workgroup_Size_X",
        "workgroup_y": "Workgroup_Size_Y", "workgroup_z": "Workgroup_Size_Z", "grid_x": "Grid_Size_X",
        "grid_y": "Grid_Size_Y", "grid_z": "Grid_Size_Z"}


def load_rows(path: str):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        cur = c.execute("select " + ", ".join(_MAP) + " from kernels")
        rows = [{_MAP[k]: v for k, v in zip(_MAP, r)} for r in cur.fetchall()]
        c.close()
    else:
        with open(path) as f:
            rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows
