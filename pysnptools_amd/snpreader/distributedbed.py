"""DistributedBed: BED data stored as per-chromosome pieces (reference
snpreader/distributedbed.py:16-207).

Storage is a local directory (the reference's ``FileCache`` cluster back-ends are out of
scope).  Layout, exactly as the reference writes it:
``chrom{c}.piece{i}of{p}.{bed,bim,fam}`` (count_A1=True BEDs), ``reader_name_list.npz`` and
``metadata.npz`` (the merged iid/sid/pos cache).  Both .npz files are read with
``allow_pickle=False``.  Pieces are SNP shards that share the iids, so the GRM of a
DistributedBed is one GPU session summing the pieces' fused decode->standardize->SYRK (and
across GPUs, one RCCL all-reduce: ``pysnptools_amd.shard.grm_pieces``).
"""
import os

import numpy as np

from pysnptools_amd.snpreader.bed import Bed
from pysnptools_amd.snpreader.snpreader import SnpReader
from pysnptools_amd.snpreader._mergesids import _MergeSIDs


class LocalCache(object):
    """Minimal local-directory storage (the reference's util/filecache/localcache.py role)."""

    def __init__(self, directory):
        self.directory = os.path.abspath(str(directory))

    def __repr__(self):
        return "LocalCache('{0}')".format(self.directory)

    def path(self, name):
        return os.path.join(self.directory, name)

    def file_exists(self, name):
        return os.path.exists(self.path(name))

    def remove(self, name):
        os.remove(self.path(name))

    @staticmethod
    def _fixup(storage):
        if isinstance(storage, LocalCache):
            return storage
        if isinstance(storage, (str, os.PathLike)):
            return LocalCache(storage)
        raise TypeError("DistributedBed storage must be a directory path (FileCache back-ends are not supported)")


def _piece_bed(storage, name, row=None):
    bed = Bed(storage.path(name), count_A1=True, skip_format_check=True)
    if row is not None:
        bed._row = row
    return bed


class DistributedBed(SnpReader):
    def __init__(self, storage):
        super(DistributedBed, self).__init__()
        self._ran_once = False
        self._storage = LocalCache._fixup(storage)
        self._merge = None

    def __repr__(self):
        return "{0}({1})".format(self.__class__.__name__, self._storage)

    def _run_once(self):
        if self._ran_once:
            return
        self._ran_once = True
        with np.load(self._storage.path("reader_name_list.npz"), allow_pickle=False) as d:
            names = np.array(d["reader_name_list"], dtype="str")
        self._merge = _MergeSIDs([_piece_bed(self._storage, str(n)) for n in names],
                                 cache_file=self._storage.path("metadata.npz"), skip_check=True)
        for reader in self._merge.reader_list:
            reader._row = self._merge.row
            reader._num_threads = None

    @property
    def row(self):
        self._run_once()
        return self._merge.row

    @property
    def col(self):
        self._run_once()
        return self._merge.col

    @property
    def col_property(self):
        self._run_once()
        return self._merge.col_property

    @property
    def pieces(self):
        """The per-piece Bed readers, in SNP order (the unit of sharding across GPUs)."""
        self._run_once()
        return list(self._merge.reader_list)

    def _read(self, iid_index_or_none, sid_index_or_none, order, dtype, force_python_only, view_ok, num_threads):
        self._run_once()
        return self._merge._read(iid_index_or_none, sid_index_or_none, order, np.dtype(dtype), force_python_only,
                                 view_ok, num_threads)

    @staticmethod
    def write(storage, snpreader, piece_per_chrom_count=1, updater=None, runner=None):
        """Split ``snpreader`` by chromosome into ``piece_per_chrom_count`` SNP pieces each and
        write them (count_A1=True) plus the metadata caches (distributedbed.py:108-207).
        Existing complete pieces are kept; ``runner`` (map_reduce) is accepted and ignored:
        pieces are encoded one after another on the GPU."""
        count_A1 = True
        storage = LocalCache._fixup(storage)
        os.makedirs(storage.directory, exist_ok=True)
        chrom_set = sorted(set(snpreader.pos[:, 0]))
        for chrom in chrom_set:
            assert chrom == chrom and chrom == int(chrom), \
                "DistributedBed.write expects all chromosomes to be integers (not '{0}')".format(chrom)
        names = []
        for chrom in chrom_set:
            chrom_reader = snpreader[:, snpreader.pos[:, 0] == chrom]
            for k in range(piece_per_chrom_count):
                start = chrom_reader.sid_count * k // piece_per_chrom_count
                stop = chrom_reader.sid_count * (k + 1) // piece_per_chrom_count
                files = ["chrom{0}.piece{1}of{2}.{3}".format(int(chrom), k, piece_per_chrom_count, sfx)
                         for sfx in ("bim", "fam", "bed")]
                exist = [storage.file_exists(f) for f in files]
                if sum(exist) < 3:
                    for f, e in zip(files, exist):
                        if e:
                            storage.remove(f)
                    Bed.write(storage.path(files[-1]), chrom_reader[:, start:stop].read(), count_A1=count_A1)
                names.append(files[-1])
        meta = storage.path("metadata.npz")
        np.savez(storage.path("reader_name_list.npz"), reader_name_list=np.array(names, dtype="S"))
        if os.path.exists(meta):
            os.remove(meta)
        _MergeSIDs([_piece_bed(storage, n) for n in names], cache_file=meta, skip_check=True)
        return DistributedBed(storage)
