! =============================================================================
! decomp_harness -- TEST INFRASTRUCTURE ONLY (the "oracle", never the product)
!
! Runs the reference's own domain decomposition on a mesh given as raw arrays:
! the unmodified framework/mpas_block_decomp.F (cells of each block from a
! graph.info.part.N file, mpas_block_decomp_cells_for_proc) and
! framework/mpas_block_creator.F (owned cells, edges and vertices, their halo
! layers and exchange lists), called in the order mpas_bootstrapping.F:171-269
! calls them, on one MPI task holding every block or under mpirun.  It dumps, per block, the
! global index of every local element (indexTo*ID, owned first, then each halo
! layer), the per-layer end counts (n*Solve fields), and the exchange lists of
! the indexTo*ID fields, which pins mpas_dycore/decomp.py (tests/test_decomp_pinned.py).
!
! Usage: decomp_harness <input_dir> <output_dir>   (or under mpirun -np P: P tasks, the blocks dealt
!        out by mpas_block_decomp.F; tasks exchange through sendList / recvList instead of copyList)
!   <input_dir>/decomp.nml  namelist /decomp/ nCells, nEdges, nVertices, maxEdges, nblocks, nHalos
!   <input_dir>/{nEdgesOnCell,cellsOnCell,edgesOnCell,verticesOnCell,cellsOnEdge,cellsOnVertex}.bin
!     int32, MPAS 1-based (Fortran memory images without the garbage slot)
!   <input_dir>/graph.info.part.<nblocks>  (what mpas_block_decomp.F reads)
! =============================================================================
program decomp_harness
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types
   use mpas_dmpar
   use mpas_log
   use mpas_block_decomp
   use mpas_block_creator
   implicit none

   character(len=256) :: indir, outdir
   integer :: nCells, nEdges, nVertices, maxEdges, nblocks, nHalos, u, i
   integer :: cs, ce, es, ee, vs, ve   ! this task's read ranges (mpas_dmpar_get_index_range)
   integer, parameter :: vertexDegree = 3
   namelist /decomp/ nCells, nEdges, nVertices, maxEdges, nblocks, nHalos

   type (domain_type), pointer :: domain
   type (block_type), pointer :: readingBlock
   type (graph) :: partial_global_graph_info
   integer, dimension(:), pointer :: local_cell_list, block_id, block_start, block_count
   type (field1dInteger), pointer :: indexToCellIDField, nEdgesOnCellField, indexToEdgeIDField, indexToVertexIDField
   type (field2dInteger), pointer :: cellsOnCellField, edgesOnCellField, verticesOnCellField, cellsOnEdgeField, &
                                     cellsOnVertexField
   type (field1dInteger), pointer :: indexToCellID_Block, nEdgesOnCell_Block, indexToEdgeID_Block, &
                                     indexToVertexID_Block, nCellsSolveField, nEdgesSolveField, nVerticesSolveField
   type (field2dInteger), pointer :: cellsOnCell_Block, verticesOnCell_Block, edgesOnCell_Block, cellsOnEdge_Block, &
                                     cellsOnVertex_Block

   call get_command_argument(1, indir)
   call get_command_argument(2, outdir)
   nHalos = 2
   open(newunit=u, file=trim(indir)//'/decomp.nml', status='old')
   read(u, nml=decomp)
   close(u)

   allocate(domain)
   allocate(domain % dminfo)
   call mpas_dmpar_init(domain % dminfo)
   allocate(domain % core)
   domain % core % coreName = 'decomp'
   call mpas_log_init(domain % logInfo, domain)
   call mpas_log_open()

   ! ---- the "read" fields (mpas_io_setup_*_block_fields): each task reads its contiguous range of
   ! cells, edges and vertices, as mpas_bootstrapping.F:171-199 does ----
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nCells, cs, ce)
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nEdges, es, ee)
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nVertices, vs, ve)
   allocate(readingBlock)
   readingBlock % domain => domain
   readingBlock % blockID = domain % dminfo % my_proc_id
   readingBlock % localBlockID = 0
   call read_field1(indexToCellIDField, '', cs, ce, nHalos)
   call read_field1(nEdgesOnCellField, 'nEdgesOnCell', cs, ce, -1, indexToCellIDField)
   call read_field2(cellsOnCellField, 'cellsOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field2(edgesOnCellField, 'edgesOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field2(verticesOnCellField, 'verticesOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field1(indexToEdgeIDField, '', es, ee, nHalos + 1)
   call read_field2(cellsOnEdgeField, 'cellsOnEdge', 2, es, ee, indexToEdgeIDField)
   call read_field1(indexToVertexIDField, '', vs, ve, nHalos + 1)
   call read_field2(cellsOnVertexField, 'cellsOnVertex', vertexDegree, vs, ve, indexToVertexIDField)

   ! ---- mpas_bootstrapping.F:207-269 ----
   partial_global_graph_info % nVertices = ce - cs + 1
   partial_global_graph_info % nVerticesTotal = nCells
   partial_global_graph_info % maxDegree = maxEdges
   partial_global_graph_info % ghostStart = nVertices + 1
   allocate(partial_global_graph_info % vertexID(ce - cs + 1))
   allocate(partial_global_graph_info % nAdjacent(ce - cs + 1))
   allocate(partial_global_graph_info % adjacencyList(maxEdges, ce - cs + 1))
   partial_global_graph_info % vertexID(:) = indexToCellIDField % array(:)
   partial_global_graph_info % nAdjacent(:) = nEdgesOnCellField % array(:)
   partial_global_graph_info % adjacencyList(:,:) = cellsOnCellField % array(:,:)
   call mpas_block_decomp_cells_for_proc(domain % dminfo, partial_global_graph_info, local_cell_list, block_id, &
                                         block_start, block_count, nblocks, .false., &
                                         trim(indir)//'/graph.info.part.', '')
   call mpas_block_creator_setup_blocks_and_0halo_cells(nHalos, domain, indexToCellID_Block, local_cell_list, &
                                                        block_id, block_start, block_count)
   call mpas_block_creator_build_0halo_cell_fields(nHalos, indexToCellIDField, nEdgesOnCellField, cellsOnCellField, &
                                                   verticesOnCellField, edgesOnCellField, indexToCellID_Block, &
                                                   nEdgesOnCell_Block, cellsOnCell_Block, verticesOnCell_Block, &
                                                   edgesOnCell_Block)
   call mpas_block_creator_build_0_and_1halo_edge_fields(nHalos, indexToEdgeIDField, cellsOnEdgeField, &
                                                         indexToCellID_Block, nEdgesOnCell_Block, edgesOnCell_Block, &
                                                         indexToEdgeID_Block, cellsOnEdge_Block, nEdgesSolveField)
   call mpas_block_creator_build_0_and_1halo_edge_fields(nHalos, indexToVertexIDField, cellsOnVertexField, &
                                                         indexToCellID_Block, nEdgesOnCell_Block, verticesOnCell_Block, &
                                                         indexToVertexID_Block, cellsOnVertex_Block, nVerticesSolveField)
   call mpas_block_creator_build_cell_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, cellsOnCell_Block, &
                                            verticesOnCell_Block, edgesOnCell_Block, nCellsSolveField)
   call mpas_block_creator_build_edge_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, nCellsSolveField, &
                                            edgesOnCell_Block, indexToEdgeID_Block, cellsOnEdge_Block, nEdgesSolveField)
   call mpas_block_creator_build_edge_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, nCellsSolveField, &
                                            verticesOnCell_Block, indexToVertexID_Block, cellsOnVertex_Block, &
                                            nVerticesSolveField)

   call dump_location('cell', indexToCellID_Block, nCellsSolveField)
   call dump_location('edge', indexToEdgeID_Block, nEdgesSolveField)
   call dump_location('vertex', indexToVertexID_Block, nVerticesSolveField)
   write(0, '(a)') 'decomp_harness: done'
   call mpas_dmpar_finalize(domain % dminfo)

contains

   ! elements s..e of a file of d1 int32 per element
   subroutine read_i(name, a, d1, s, e)
      character(len=*), intent(in) :: name
      integer, intent(in) :: d1, s, e
      integer, intent(out) :: a(d1 * (e - s + 1))
      integer :: uu
      open(newunit=uu, file=trim(indir)//'/'//name//'.bin', access='stream', form='unformatted', status='old')
      read(uu, pos=int(4, 8) * int(d1, 8) * int(s - 1, 8) + 1) a
      close(uu)
   end subroutine read_i

   ! a 1-d read field of elements s..e; name '' = the index field itself (s..e), which owns the
   ! exchange lists
   subroutine read_field1(f, name, s, e, nlayers, owner)
      type (field1dInteger), pointer :: f
      character(len=*), intent(in) :: name
      integer, intent(in) :: s, e, nlayers
      type (field1dInteger), pointer, optional :: owner
      integer :: j, n
      n = e - s + 1
      allocate(f)
      allocate(f % array(n))
      if (len(name) == 0) then
         f % array = [(j, j = s, e)]
         call mpas_dmpar_init_multihalo_exchange_list(f % sendList, nlayers)
         call mpas_dmpar_init_multihalo_exchange_list(f % recvList, nlayers)
         call mpas_dmpar_init_multihalo_exchange_list(f % copyList, nlayers)
      else
         call read_i(name, f % array, 1, s, e)
         f % sendList => owner % sendList
         f % recvList => owner % recvList
         f % copyList => owner % copyList
      end if
      f % dimSizes(1) = n
      f % block => readingBlock
      nullify(f % next)
   end subroutine read_field1

   subroutine read_field2(f, name, d1, s, e, owner)
      type (field2dInteger), pointer :: f
      character(len=*), intent(in) :: name
      integer, intent(in) :: d1, s, e
      type (field1dInteger), pointer :: owner
      integer :: n
      n = e - s + 1
      allocate(f)
      allocate(f % array(d1, n))
      call read_i(name, f % array, d1, s, e)
      f % dimSizes(1) = d1
      f % dimSizes(2) = n
      f % block => readingBlock
      f % sendList => owner % sendList
      f % recvList => owner % recvList
      f % copyList => owner % copyList
      nullify(f % next)
   end subroutine read_field2

   ! per block (global block id i): <out>/block<i>/<loc>_index.bin (global ids, local order), <loc>_solve.bin (end of
   ! the owned elements and of each halo layer), and every exchange list node of the index field:
   ! <loc>_<kind>_<layer>.bin = records (endPointID, nList, srcList(nList), destList(nList))
   subroutine dump_location(loc, idx, solve)
      character(len=*), intent(in) :: loc
      type (field1dInteger), pointer :: idx, solve
      type (field1dInteger), pointer :: fi, fs
      type (mpas_multihalo_exchange_list), pointer :: ml
      type (mpas_exchange_list), pointer :: node
      character(len=320) :: dir
      integer :: uu, kind, layer
      character(len=4), dimension(3), parameter :: kinds = ['send', 'recv', 'copy']
      fi => idx
      fs => solve
      do while (associated(fi))
         write(dir, '(a,a,i0)') trim(outdir), '/block', fi % block % blockID
         call execute_command_line('mkdir -p '//trim(dir))
         open(newunit=uu, file=trim(dir)//'/'//loc//'_index.bin', access='stream', form='unformatted', status='replace')
         write(uu) fi % array(1:fi % dimSizes(1))
         close(uu)
         open(newunit=uu, file=trim(dir)//'/'//loc//'_solve.bin', access='stream', form='unformatted', status='replace')
         write(uu) fs % array(1:fs % dimSizes(1))
         close(uu)
         do kind = 1, 3
            if (kind == 1) ml => fi % sendList
            if (kind == 2) ml => fi % recvList
            if (kind == 3) ml => fi % copyList
            do layer = 1, size(ml % halos)
               write(dir, '(a,a,i0,a,a,a,a,a,i0,a)') trim(outdir), '/block', fi % block % blockID, '/', loc, '_', &
                     kinds(kind), '_', layer, '.bin'
               open(newunit=uu, file=trim(dir), access='stream', form='unformatted', status='replace')
               node => ml % halos(layer) % exchList
               do while (associated(node))
                  write(uu) node % endPointID, node % nList, node % srcList(1:node % nList), node % destList(1:node % nList)
                  node => node % next
               end do
               close(uu)
            end do
         end do
         fi => fi % next
         fs => fs % next
      end do
   end subroutine dump_location

end program decomp_harness
